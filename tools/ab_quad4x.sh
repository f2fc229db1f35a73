# Same-box A/B for the 4x quad kernel and compact leaves (tools/_old = previous HEAD).
set -e
run() { timeout -k 10 200 python3 tools/ab_old_new.py "$@" 2>&1 | grep " ms" | tail -1; }
run old quad c3
run new quad c3 fused
run new quad c3 compact
run new sector c3
run new inline c3 compact
run new quad c1 fused
run new quad c1 compact
python3 -c "
import numpy as np
a = np.load('/tmp/ab_old_quad_c3_fused.npy')
for k in ('new_quad_c3_fused', 'new_quad_c3_compact', 'new_sector_c3_fused', 'new_inline_c3_compact'):
    print(k, 'identical to old quad', np.array_equal(a, np.load('/tmp/ab_' + k + '.npy')))
print('c1 compact == fused', np.array_equal(np.load('/tmp/ab_new_quad_c1_fused.npy'), np.load('/tmp/ab_new_quad_c1_compact.npy')))
"
