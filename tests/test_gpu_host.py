"""Host-pointer search calls (csrc/host_stage.hpp): pinned staging slots, chunked H2D /
kernel / D2H over three streams, host-side 2-bit packing for PREFIX with m <= 32.

Bar: bit-identical to the same queries through device pointers (themselves checked against
the oracle elsewhere) for batches that span many chunks, fixed and ragged, every mode
(bytes, packed on the host, the caller's packed words); a code > 3 anywhere fails the whole
call with EINVAL; concurrent host calls on one index each get their own slots.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch

    import sas_amd
    n = 3_000_017
    t = sas_amd.random_string(n, seed=77)
    idx = sas_amd.SaNaive.build(torch.from_numpy(t).cuda(), prefix=12)
    return sas_amd, torch, t, idx


def dev_search(torch, idx, qb, m, algo):
    out = idx.search_fixed(torch.from_numpy(qb).cuda(), m, algo=algo)
    torch.cuda.synchronize()
    return out.cpu().numpy().astype(np.uint64)


def fixed_queries(t, nq, m, seed):
    rng = np.random.default_rng(seed)
    offs = rng.integers(0, len(t) - m, nq)
    qb = t[offs[:, None] + np.arange(m)[None, :]].reshape(-1).copy()
    qb[: (nq // 8) * m] = rng.integers(0, 4, (nq // 8) * m, dtype=np.uint8)
    return qb


@pytest.mark.parametrize("m", [1, 7, 16, 31, 32])
def test_prefix_host_packing(env, m):
    """PREFIX from host bytes, m <= 32: packed 2-bit on the host (several 2^19-query
    chunks at m = 32), equal to the device run; probes too."""
    sas, torch, t, idx = env
    nq = 1_300_000 if m == 32 else 60_000
    qb = fixed_queries(t, nq, m, m)
    expect = dev_search(torch, idx, qb, m, "prefix")
    got, pr = idx.search_fixed(qb, m, algo="prefix", probes=True)
    assert np.array_equal(got, expect)
    _, dpr = idx.search_fixed(torch.from_numpy(qb).cuda(), m, algo="prefix", probes=True)
    assert np.array_equal(pr, dpr.cpu().numpy().astype(np.uint32))


def test_byte_staging_many_chunks(env):
    """PLAIN / QUAD from host bytes (16 MiB chunks): m = 100 fixed over > 3 chunks."""
    sas, torch, t, idx = env
    m, nq = 100, 700_000
    qb = fixed_queries(t, nq, m, 5)
    for algo in ("plain", "quad"):
        assert np.array_equal(idx.search_fixed(qb, m, algo=algo), dev_search(torch, idx, qb, m, algo)), algo


def test_ragged_staging_many_chunks(env):
    """Ragged host queries with gaps and out-of-order offsets, > 16 MiB of bytes: gathered
    chunk by chunk, equal to the device run over the same buffer."""
    sas, torch, t, idx = env
    rng = np.random.default_rng(9)
    nq = 400_000
    lens = rng.integers(0, 200, nq).astype(np.uint32)
    starts = rng.integers(0, len(t) - 200, nq)
    buf = np.concatenate([t[s:s + l] for s, l in zip(starts, lens)] + [np.zeros(64, np.uint8)])
    off = np.zeros(nq, np.uint64)
    off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    perm = rng.permutation(nq)  # offsets out of order
    off, lens = off[perm], lens[perm]
    d = idx.search_batch(torch.from_numpy(buf).cuda(), torch.from_numpy(off.view(np.int64)).cuda(),
                         torch.from_numpy(lens.view(np.int32)).cuda(), algo="plain")
    torch.cuda.synchronize()
    got = idx.search_batch(buf, off, lens, algo="plain")
    assert np.array_equal(got, d.cpu().numpy().astype(np.uint64))


def test_packed_words_host(env):
    """sas_search_packed with host words (the caller's packing) == device words."""
    sas, torch, t, idx = env
    m, nq = 32, 600_000
    qb = fixed_queries(t, nq, m, 3)
    w = sas.SaNaive.pack_queries(torch.from_numpy(qb).cuda(), m)
    torch.cuda.synchronize()
    hw = w.cpu().numpy().view(np.uint64)
    assert np.array_equal(idx.search_packed(hw, m), dev_search(torch, idx, qb, m, "prefix"))


def test_host_invalid_codes(env):
    """A code > 3 in any chunk fails the call (packed and byte modes)."""
    from sas_amd._lib import SasError
    sas, torch, t, idx = env
    for m, algo in ((32, "prefix"), (20, "prefix"), (40, "plain")):
        qb = fixed_queries(t, 1_100_000 if m == 32 else 50_000, m, 1)
        qb[len(qb) - 3] = 4
        with pytest.raises(SasError):
            idx.search_fixed(qb, m, algo=algo)
        qb[len(qb) - 3] = 2  # the index and its slots stay usable
        assert np.array_equal(idx.search_fixed(qb, m, algo=algo), dev_search(torch, idx, qb, m, algo))


def test_concurrent_host_calls(env):
    """Four threads searching host arrays on one index at once."""
    sas, torch, t, idx = env
    m = 32
    batches = [fixed_queries(t, 300_000, m, 20 + k) for k in range(4)]
    expect = [dev_search(torch, idx, b, m, "prefix") for b in batches]
    got, errs = {}, []

    def run(k):
        try:
            algo = "prefix" if k % 2 == 0 else "quad"
            got[k] = (algo, idx.search_fixed(batches[k], m, algo=algo))
        except Exception as e:
            errs.append(repr(e))
    th = [threading.Thread(target=run, args=(k,)) for k in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not errs, errs
    for k in range(4):
        assert np.array_equal(got[k][1], expect[k]), k


def test_ranges_host_pipeline(env):
    """sas_search_range(_fixed) from host arrays runs through the staging pipeline (chunks
    of at most half the slot's positions: lo and hi share them): fixed m = 32 over several
    chunks and ragged lengths equal the device-pointer ranges; a code > 3 is EINVAL."""
    sas, torch, t, idx = env
    m, nq = 32, 1_300_000
    qb = fixed_queries(t, nq, m, 9)
    lo, hi = idx.search_range_fixed(qb, m)
    dlo, dhi = idx.search_range_fixed(torch.from_numpy(qb).cuda(), m)
    assert np.array_equal(lo, dlo.cpu().numpy().astype(np.uint64))
    assert np.array_equal(hi, dhi.cpu().numpy().astype(np.uint64))
    assert (hi[nq // 8:] > lo[nq // 8:]).all()  # positives occur
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 120, 400_000).astype(np.uint32)
    offs = rng.integers(0, len(t) - 130, len(lens)).astype(np.uint64)
    buf = np.concatenate([t, np.zeros(64, np.uint8)])
    lo, hi = idx.search_range(buf, offs, lens)
    dlo, dhi = idx.search_range(torch.from_numpy(buf).cuda(), torch.from_numpy(offs.astype(np.int64)).cuda(),
                                torch.from_numpy(lens.astype(np.int32)).cuda())
    assert np.array_equal(lo, dlo.cpu().numpy().astype(np.uint64))
    assert np.array_equal(hi, dhi.cpu().numpy().astype(np.uint64))
    bad = qb.copy()
    bad[777 * m + 5] = 9
    with pytest.raises(sas.SasError):
        idx.search_range_fixed(bad, m)
