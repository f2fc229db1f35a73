#!/bin/bash
# Round-5 kernel statistics (GPU box): rocprofv3 --kernel-trace --stats over the default bench
# without the host-buffer pass and configs[3]/[4] (the headline k_sa_prefix2, every variant,
# both configs[1] figures, lcp_long and the u32 path), then the per-grid summary of the search
# kernels (tools/kt_by_grid.py) and rocprofv3's own kernel_stats.csv.
# usage: tools/prof_r5.sh [outdir]
set -o pipefail
out=${1:-gpurun_out/prof6}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- python3 bench.py \
    --no-e2e --no-c3 --no-c4 --no-cpu --detail "$out/kt_detail.json" \
    > "$out/kt_bench.json" 2> "$out/kt_bench.err" || exit $?
python3 tools/kt_by_grid.py "$out/kt/run_kernel_trace.csv" "$out/kt/kernel_stats_by_grid.csv" k_sa_ k_sst_ || exit $?
find "$out/kt" -name '*kernel_trace.csv' -delete
python3 - "$out" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1] + '/kt/kernel_stats_by_grid.csv')):
    if int(r['Calls']) >= 10:
        print(r['Kernel_Name'][:70], r['Grid'], r['Calls'], round(float(r['AverageNs']) / 1000, 1),
              round(float(r['MedianNs']) / 1000, 1))
PY
