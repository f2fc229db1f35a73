#!/bin/bash
# Round-5 kernel statistics of configs[3] and configs[4] (GPU box): rocprofv3 --kernel-trace
# --stats over `bench.py --workload c3` (bucket lines + the rank-ordered cross-check) and over
# the default bench's configs[4] step alone (--no-* everything else), then the per-grid summary.
# usage: tools/prof_r5_c34.sh [outdir]
set -o pipefail
out=${1:-gpurun_out/prof5_c34}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/c3" -o run -- python3 bench.py \
    --workload c3 > "$out/c3_bench.json" 2> "$out/c3_bench.err" || exit $?
python3 tools/kt_by_grid.py "$out/c3/run_kernel_trace.csv" "$out/c3/kernel_stats_by_grid.csv" k_sa_ || exit $?
find "$out/c3" -name '*kernel_trace.csv' -delete
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/c4" -o run -- python3 bench.py \
    --no-cpu --no-c3 --no-sst --no-e2e --no-lcp-long --variants= --c1-deep-levels 0 --steps 3 --warmup 1 \
    --detail "$out/c4_detail.json" > "$out/c4_bench.json" 2> "$out/c4_bench.err" || exit $?
python3 tools/kt_by_grid.py "$out/c4/run_kernel_trace.csv" "$out/c4/kernel_stats_by_grid.csv" k_ || exit $?
find "$out/c4" -name '*kernel_trace.csv' -delete
