"""Host-side 2-bit query packing (csrc/host_stage.hpp, the staging pipeline's packer, exposed
as sas_pack_queries on host arrays): the AVX2 path (m = 32), the BMI2 path (SAS_NO_AVX2=1, in
a child process) and the portable path all equal a numpy restatement of the word format
(first char in bits 63..62, zero padded), and a code > 3 is EINVAL.  CPU only: no GPU call."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def np_pack(qb, m):
    q = qb.reshape(-1, m).astype(np.uint64)
    w = np.zeros(len(q), np.uint64)
    for j in range(m):
        w |= q[:, j] << np.uint64(62 - 2 * j)
    return w


@pytest.mark.parametrize("m", [1, 7, 16, 31, 32])
def test_host_pack_matches_numpy(m):
    import sas_amd
    rng = np.random.default_rng(m)
    qb = rng.integers(0, 4, 100_003 * m, dtype=np.uint8)
    assert np.array_equal(sas_amd.SaNaive.pack_queries(qb, m), np_pack(qb, m))
    bad = qb.copy()
    bad[77 * m + m // 2] = 4
    with pytest.raises(sas_amd.SasError):
        sas_amd.SaNaive.pack_queries(bad, m)


def test_host_pack_without_avx2():
    code = ("import numpy as np, sys; sys.path.insert(0, 'tests'); from test_host_pack import np_pack; "
            "import sas_amd; rng = np.random.default_rng(5); qb = rng.integers(0, 4, 50_001 * 32, dtype=np.uint8); "
            "assert np.array_equal(sas_amd.SaNaive.pack_queries(qb, 32), np_pack(qb, 32)); print('ok')")
    env = dict(os.environ, SAS_NO_AVX2="1", PYTHONPATH=os.path.join(ROOT, "suffix-array-searching_amd") + ":" + ROOT)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]
