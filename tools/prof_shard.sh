#!/bin/bash
# Kernel-level breakdown of the sharded step at world size 1 (run on the GPU box).
set -o pipefail
out=gpurun_out/prof_shard
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$out/kt" -o run -- python3 bench.py --mode shard --no-c3 --no-c4 --no-cpu --no-e2e --variants "" --steps 10 > "$out/shard.json" 2> "$out/shard.err" || exit $?
python3 tools/kt_by_grid.py "$out/kt/run_kernel_trace.csv" "$out/kt/kernel_stats_by_grid.csv" || exit $?
find "$out/kt" -name '*_trace.csv' -delete
exit 0
