set -o pipefail
mkdir -p gpurun_out/s1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_shard.py tests/test_gpu_sa.py::test_route_pack > gpurun_out/s1/tests.log 2>&1 || { tail -30 gpurun_out/s1/tests.log; exit 1; }
tail -3 gpurun_out/s1/tests.log
timeout -k 10 300 python -u bench.py --mode shard --no-c3 --no-c4 --no-cpu --no-e2e --variants "" --steps 20 > gpurun_out/s1/shard.json 2> gpurun_out/s1/shard.err || { tail -20 gpurun_out/s1/shard.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/s1/shard.json'));print(d['value'],d['ms_per_step'])"
bash tools/prof_shard.sh && head -15 gpurun_out/prof_shard/kt/kernel_stats_by_grid.csv
