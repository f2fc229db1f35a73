# configs[3] shape at n = 2^34 (compact quad leaves): bench line, rocprofv3 kernel stats,
# and the PMC passes for roofline.traffic.  Run on the GPU box.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c3
timeout -k 10 400 python3 bench.py --workload c3 --steps 3 --warmup 1 > gpurun_out/c3/bench.json 2> gpurun_out/c3/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3/kt -o run -- python3 bench.py --no-cpu --workload c3 --steps 3 --warmup 1 > gpurun_out/c3/kt.json 2> gpurun_out/c3/kt.err
bash tools/pmc_pass.sh gpurun_out/c3/pmc --workload c3 --steps 2 --warmup 1
