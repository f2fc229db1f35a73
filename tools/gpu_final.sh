#!/bin/bash
# End-of-session GPU check (GPU box): -m gpu suite, smoke(), default bench, kernel-trace profile.
set -o pipefail
bash tools/gpu_full.sh || exit $?
bash tools/prof_r2.sh kt || exit $?
python3 - <<'PY'
import csv, json
for r in csv.DictReader(open('gpurun_out/prof/kt/kernel_stats_by_grid.csv')):
    if r['Grid'] == '524288x1x1' or 'tagged' in r['Kernel_Name']:
        print(r['Kernel_Name'][:60], r['Grid'], r['Calls'], round(float(r['AverageNs']) / 1000, 1))
PY
