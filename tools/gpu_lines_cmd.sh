set -o pipefail
mkdir -p gpurun_out/lines
timeout -k 10 600 python -u -m pytest tests/test_gpu_tagged.py -x -q --timeout 300 --timeout-method thread > gpurun_out/lines/test.log 2>&1 || { tail -30 gpurun_out/lines/test.log; exit 1; }
tail -2 gpurun_out/lines/test.log
AB_ROUNDS=${AB_ROUNDS:-2} AB_PKGS=${AB_PKGS:-suffix-array-searching_amd} NO_PMC=1 bash tools/gpu_lines_ab.sh
