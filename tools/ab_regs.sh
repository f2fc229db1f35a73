set -e
run() { timeout -k 10 200 python3 tools/ab_old_new.py "$@" 2>&1 | grep " ms" | tail -1; }
for r in 1 2 3; do
run new quad c3 fused
run old1 quad c3 fused
run old2 quad c3 fused
done
run new quad c3 compact
run old1 quad c3 compact
run old2 quad c3 compact
python3 -c "
import numpy as np
a = np.load('/tmp/ab_new_quad_c3_fused.npy')
print('regs1 identical', np.array_equal(a, np.load('/tmp/ab_old1_quad_c3_fused.npy')), np.array_equal(a, np.load('/tmp/ab_old1_quad_c3_compact.npy')))
"
