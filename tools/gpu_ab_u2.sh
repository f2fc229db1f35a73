#!/bin/bash
# headline kernel: same-box A/B of the two-queries-per-pair variant (tools/_var_u2)
set -o pipefail
out=gpurun_out/u2
mkdir -p "$out"
for r in 1 2; do
  for v in main u2; do
    if [ $v = main ]; then pk=suffix-array-searching_amd; else pk=tools/_var_u2/suffix-array-searching_amd; fi
    AB_MODES=16d AB_PKG=$pk timeout -k 10 300 python3 -u tools/ab_prefix.py > "$out/ab_${v}_$r.txt" 2> "$out/ab_${v}_$r.err" || { tail -20 "$out/ab_${v}_$r.err"; exit 1; }
    echo "$v round $r: $(tail -3 $out/ab_${v}_$r.txt)"
  done
done
