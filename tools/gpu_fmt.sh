#!/bin/bash
# Round-3 line format (20 slots, second text copy): tagged parity tests, same-box A/B against
# the previous format (tools/_var_old, built by tools/mk_variant_git.sh), the configs[3]
# full-size test, then the c3 PMC passes.  Stops at the first failing step.
set -o pipefail
out=gpurun_out/fmt
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_tagged.py -x -v --timeout 300 --timeout-method thread > "$out/tagged.log" 2>&1 || { tail -40 "$out/tagged.log"; exit 1; }
tail -2 "$out/tagged.log"
AB_TAG=new timeout -k 10 420 python3 -u tools/ab_lines_fmt.py > "$out/ab_new.txt" 2> "$out/ab_new.err" || { tail -20 "$out/ab_new.err"; cat "$out/ab_new.txt"; exit 1; }
cat "$out/ab_new.txt"
if [ -d tools/_var_old ]; then
  AB_TAG=old AB_PKG=tools/_var_old/suffix-array-searching_amd timeout -k 10 420 python3 -u tools/ab_lines_fmt.py > "$out/ab_old.txt" 2> "$out/ab_old.err" || { tail -20 "$out/ab_old.err"; exit 1; }
  cat "$out/ab_old.txt"
  AB_TAG=new2 AB_ROUNDS=2 timeout -k 10 420 python3 -u tools/ab_lines_fmt.py > "$out/ab_new2.txt" 2> "$out/ab_new2.err" || { tail -20 "$out/ab_new2.err"; exit 1; }
  cat "$out/ab_new2.txt"
  python3 -c "
import numpy as np
a, b = np.load('/tmp/ab_lines_new.npy'), np.load('/tmp/ab_lines_old.npy')
print('new format == old format positions:', bool(np.array_equal(a, b)))
" | tee "$out/ab_cmp.txt"
fi
[ -n "$NO_C3TEST" ] || { timeout -k 10 900 python3 -u -m pytest tests/test_gpu_c3.py -x -v --timeout 800 --timeout-method thread > "$out/c3test.log" 2>&1 || { tail -40 "$out/c3test.log"; exit 1; }; tail -2 "$out/c3test.log"; }
[ -n "$NO_PMC" ] || bash tools/pmc_r3.sh c3
