#!/bin/bash
# bucket-line kernel: same-box A/B of 4 (main) against 5 (tools/_var_lb5) waves per SIMD
set -o pipefail
out=gpurun_out/lb
mkdir -p "$out"
for v in main lb5 main2 lb5b; do
  case $v in main*) pk=suffix-array-searching_amd ;; *) pk=tools/_var_lb5/suffix-array-searching_amd ;; esac
  AB_TAG=$v AB_PKG=$pk AB_ROUNDS=2 timeout -k 10 420 python3 -u tools/ab_lines_fmt.py > "$out/ab_$v.txt" 2> "$out/ab_$v.err" || { tail -20 "$out/ab_$v.err"; exit 1; }
  cat "$out/ab_$v.txt"
done
python3 -c "
import numpy as np
a = np.load('/tmp/ab_lines_main.npy')
print('identical positions:', all(np.array_equal(a, np.load(f'/tmp/ab_lines_{t}.npy')) for t in ('lb5', 'main2', 'lb5b')))
" | tee "$out/ab_cmp.txt"
