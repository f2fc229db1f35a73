set -e
for w in old new old new; do timeout -k 10 200 python3 tools/ab_old_new.py $w quad c1 2>&1 | grep " ms" | tail -1; done
python3 -c "import numpy as np; print('identical', np.array_equal(np.load('/tmp/ab_old_quad_c1.npy'), np.load('/tmp/ab_new_quad_c1.npy')))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in new; do
  timeout -k 10 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/tlb_$w -o run -- python3 tools/ab_old_new.py $w quad c1 > /dev/null 2>&1
done
