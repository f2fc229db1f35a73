set -o pipefail
mkdir -p gpurun_out/lines
timeout -k 10 600 python -u -m pytest tests/test_gpu_tagged.py -x -q --timeout 300 --timeout-method thread > gpurun_out/lines/test.log 2>&1 || { tail -30 gpurun_out/lines/test.log; exit 1; }
tail -2 gpurun_out/lines/test.log
if [ -n "$AB_PKGS" ]; then AB_ROUNDS=${AB_ROUNDS:-2} NO_PMC=1 bash tools/gpu_lines_ab.sh || exit 1; fi
if [ -n "$WITH_TAGGED" ]; then timeout -k 10 600 python3 -u tools/ab_c3_lines.py > gpurun_out/lines/ab_tagged.txt 2> gpurun_out/lines/ab_tagged.err || { tail -20 gpurun_out/lines/ab_tagged.err; exit 1; }; cat gpurun_out/lines/ab_tagged.txt; fi
