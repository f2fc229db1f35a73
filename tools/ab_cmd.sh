set -e
for a in "stree c3" "stree c1"; do
  set -- $a
  timeout -k 10 200 python3 tools/ab_old_new.py old $1 $2 2>&1 | grep " ms" | tail -1
  timeout -k 10 200 python3 tools/ab_old_new.py new $1 $2 2>&1 | grep " ms" | tail -1
  python3 -c "import numpy as np,sys; print('identical', np.array_equal(np.load('/tmp/ab_old_$1_$2.npy'), np.load('/tmp/ab_new_$1_$2.npy')))"
done
