#!/bin/bash
# Round-4 kernel statistics (GPU box): rocprofv3 --kernel-trace --stats over the default bench
# without the host-buffer pass, the prefix_packed variant, configs[4] (all three launch
# k_sa_prefix2 on the headline's grid) and the 30-level PLAIN index (k_sa_binary on the c1
# grid), then the per-grid summary of the search kernels.  usage: tools/prof_r4.sh [outdir]
set -o pipefail
out=${1:-gpurun_out/prof4}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- python3 bench.py \
    --no-e2e --no-c4 --c1-deep-levels 0 --detail "$out/kt_detail.json" \
    --variants plain,plain_range,llcp,stree,sector,quad,inline,interp,interp_range \
    > "$out/kt_bench.json" 2> "$out/kt_bench.err" || exit $?
python3 tools/kt_by_grid.py "$out/kt/run_kernel_trace.csv" "$out/kt/kernel_stats_by_grid.csv" k_sa_ || exit $?
find "$out/kt" -name '*kernel_trace.csv' -delete
python3 - "$out" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1] + '/kt/kernel_stats_by_grid.csv')):
    if r['Grid'] in ('524288', '524288x1x1') or 'tagged' in r['Kernel_Name']:
        print(r['Kernel_Name'][:70], r['Grid'], r['Calls'], round(float(r['AverageNs']) / 1000, 1))
PY
