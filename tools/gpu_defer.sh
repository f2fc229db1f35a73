#!/bin/bash
# two-pass bucket-line calls and the offsets prefetch: tagged parity tests, then same-box A/B
# (in-tree library with SAS_TL_DEFER=1 / 0, tools/_var_nopf without the prefetch)
set -o pipefail
out=gpurun_out/defer
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_tagged.py -x -v --timeout 300 --timeout-method thread > "$out/tagged.log" 2>&1 || { tail -40 "$out/tagged.log"; exit 1; }
tail -2 "$out/tagged.log"
run() {  # tag, env...
  local t=$1; shift
  env "$@" AB_TAG=$t AB_ROUNDS=2 timeout -k 10 420 python3 -u tools/ab_lines_fmt.py > "$out/ab_$t.txt" 2> "$out/ab_$t.err" || { tail -20 "$out/ab_$t.err"; return 1; }
  cat "$out/ab_$t.txt"
}
run pf_defer1 SAS_TL_DEFER=1 || exit 1
run pf_defer0 SAS_TL_DEFER=0 || exit 1
run nopf_defer0 SAS_TL_DEFER=0 AB_PKG=tools/_var_nopf/suffix-array-searching_amd || exit 1
run nopf_defer1 SAS_TL_DEFER=1 AB_PKG=tools/_var_nopf/suffix-array-searching_amd || exit 1
run pf_defer1b SAS_TL_DEFER=1 || exit 1
python3 -c "
import numpy as np
a = np.load('/tmp/ab_lines_pf_defer1.npy')
print('identical positions:', all(np.array_equal(a, np.load(f'/tmp/ab_lines_{t}.npy')) for t in ('pf_defer0', 'nopf_defer0', 'nopf_defer1', 'pf_defer1b')))
" | tee "$out/ab_cmp.txt"
