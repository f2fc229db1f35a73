"""GPU parity of the suffix-array path (libsas_amd.so via the C ABI) against the
oracle.  Bar: bit-exact positions for every algorithm.

* definition fixtures (tests/golden/sa_definition.json): SA, LCP, positions;
* C0 shape (1 MiB ChaCha8 text, 10^4 len-16 queries) vs the oracle's
  restated binary_search (sas/sa_search.rs:98-112) on the oracle-built SA;
* larger texts: GPU-built SA checked by the reference's adjacency assertion
  (sas/sa_search.rs:36-38) on the CPU, then positions vs the oracle;
* edge cases: empty / over-long / above-all queries, text-end suffixes,
  invalid codes, m > 256 (beyond the register-resident query words).
"""
import json
import os

import numpy as np
import pytest

from oracle import pyoracle as O

pytestmark = pytest.mark.gpu

ALGOS = ("plain", "lcp", "stree", "sector", "quad", "inline", "llcp", "prefix", "interp", "stree_llcp", "quad_llcp")


@pytest.fixture(scope="module")
def sas():
    import sas_amd
    return sas_amd


@pytest.fixture(scope="module")
def sadef(golden_dir):
    return json.load(open(os.path.join(golden_dir, "sa_definition.json")))


def oracle_positions(t, sa, qbuf, off, lens, threads=8):
    tp = O.padded(t)
    qb = np.concatenate([qbuf, np.zeros(64, np.uint8)])
    pos, _ = O.search_many(tp, len(t), sa, qb, off, lens, "binary_search", threads)
    return pos


def pack(qs):
    lens = np.array([len(q) for q in qs], np.uint32)
    off = np.zeros(len(qs), np.uint64)
    if len(qs) > 1:
        off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = np.concatenate([np.asarray(q, np.uint8) for q in qs] + [np.zeros(64, np.uint8)])
    return buf, off, lens


def test_definition_fixtures(sas, sadef):
    for c in sadef["cases"]:
        t = np.array(c["text"], np.uint8)
        idx = sas.SaNaive.build(t, lcp=True, stree=True, verify=True)
        assert idx.suffix_array().tolist() == c["sa"], c["name"]
        lcp = O.kasai_lcp(t, np.array(c["sa"], np.uint32))
        assert np.array_equal(idx.lcp_array(), lcp), c["name"]
        buf, off, lens = pack([q["q"] for q in c["queries"]])
        expect = np.array([q["pos"] for q in c["queries"]], np.uint64)
        for algo in ALGOS:
            got, probes = idx.search_batch(buf, off, lens, algo=algo, probes=True)
            assert np.array_equal(got, expect), (c["name"], algo, np.nonzero(got != expect))
        # caller-supplied SA path
        idx2 = sas.SaNaive.build(t, sa=np.array(c["sa"], np.uint32), lcp=False, stree=True, verify=True)
        got = idx2.search_batch(buf, off, lens, algo="stree")
        assert np.array_equal(got, expect)


def test_no_lds_top_same(sas, sadef):
    from sas_amd import _lib
    c = [c for c in sadef["cases"] if c["name"] == "random_4096"][0]
    t = np.array(c["text"], np.uint8)
    idx = sas.SaNaive.build(t)
    buf, off, lens = pack([q["q"] for q in c["queries"]])
    expect = np.array([q["pos"] for q in c["queries"]], np.uint64)
    for algo in ("plain", "lcp", "llcp"):
        got = idx.search_batch(buf, off, lens, algo=algo, flags=_lib.SAS_NO_LDS_TOP)
        assert np.array_equal(got, expect)


def test_gen_text_bit_exact(sas):
    for n in (1, 15, 16, 17, 1000, (1 << 20) + 3):
        assert np.array_equal(sas.random_string(n), O.random_string(n)), n


def test_c0_config_parity(sas):
    """configs[0]: 1 MiB random ACGT text, 10^4 length-16 queries."""
    n, nq, m = 1 << 20, 10_000, 16
    t = sas.random_string(n)
    sa = O.build_sa(t)
    idx = sas.SaNaive.build(t, lcp=True, stree=True)
    assert np.array_equal(idx.suffix_array(), sa)
    off, lens, _ = sas.random_queries(n, nq, len_lo=m, len_hi=m + 1)
    qbytes = np.concatenate([t[o:o + m] for o in off.astype(np.int64)])
    expect = oracle_positions(t, sa, qbytes, np.arange(nq, dtype=np.uint64) * m, np.full(nq, m, np.uint32))
    for algo in ALGOS:
        got, probes = idx.search_fixed(qbytes, m, algo=algo, probes=True)
        assert np.array_equal(got, expect), algo
        if algo == "plain":
            assert (probes <= 21).all() and (probes >= 20).all()  # ilog2(n)+1 lockstep, l<r probes only
    # every positive query's answer is an occurrence of it
    tp = O.padded(t)
    got = idx.search_fixed(qbytes, m, algo="stree")
    occ = np.stack([tp[p:p + m] for p in got.astype(np.int64)])
    assert np.array_equal(occ.reshape(-1), qbytes)


@pytest.mark.parametrize("n", [1 << 16, 3_000_017, 1 << 24])
def test_random_text_mixed_queries(sas, n):
    rng = np.random.default_rng(n)
    t = sas.random_string(n, seed=n)
    idx = sas.SaNaive.build(t, lcp=True, stree=True, verify=True)
    sa = idx.suffix_array()
    assert O.check_sa(t, sa) == 0  # sas/sa_search.rs:36-38 + permutation, on the CPU
    nq = 20_000
    off, lens, _ = sas.random_queries(n, nq, seed=7, margin=256, len_lo=8, len_hi=257)  # configs[3] shape
    qs = [t[o:o + l] for o, l in zip(off.astype(np.int64), lens.astype(np.int64))]
    qs += [rng.integers(0, 4, rng.integers(0, 70), dtype=np.uint8) for _ in range(2000)]  # negatives
    qs += [np.concatenate([t[n - k:], np.zeros(5, np.uint8)]) for k in (1, 3, 31, 32, 33)]  # A7 edge
    qs += [t[n - k:] for k in (1, 2, 16, 40)]
    buf, qo, ql = pack(qs)
    expect = oracle_positions(t, sa, buf[:-64], qo, ql)
    for algo in ALGOS:
        got = idx.search_batch(buf, qo, ql, algo=algo)
        bad = np.nonzero(got != expect)[0]
        assert len(bad) == 0, (algo, bad[:10], [qs[i] for i in bad[:3]])


def test_repetitive_texts(sas):
    """Long repeats force doubling rounds, long tie runs in the S-tree leaves and
    multi-word compares."""
    rng = np.random.default_rng(3)
    blk = rng.integers(0, 4, 5000, dtype=np.uint8)
    texts = {
        "all_A": np.zeros(100_000, np.uint8),
        "period_7": np.tile(rng.integers(0, 4, 7, dtype=np.uint8), 30_000),
        "repeats": np.concatenate([blk, rng.integers(0, 4, 100, dtype=np.uint8), blk, blk[:3000], blk]),
    }
    for name, t in texts.items():
        idx = sas.SaNaive.build(t, lcp=True, stree=True, verify=True)
        sa = O.build_sa(t)
        assert np.array_equal(idx.suffix_array(), sa), name
        assert np.array_equal(idx.lcp_array(), O.kasai_lcp(t, sa)), name
        n = len(t)
        qs = [t[o:o + l] for o, l in zip(rng.integers(0, n - 600, 3000), rng.integers(1, 600, 3000))]
        qs += [np.concatenate([t[o:o + 40], [3]]).astype(np.uint8) for o in rng.integers(0, n - 50, 200)]
        qs += [t[:300], np.zeros(301, np.uint8), np.full(10, 3, np.uint8), np.zeros(0, np.uint8)]
        buf, qo, ql = pack(qs)
        expect = oracle_positions(t, sa, buf[:-64], qo, ql)
        for algo in ALGOS:
            got = idx.search_batch(buf, qo, ql, algo=algo)
            assert np.array_equal(got, expect), (name, algo)


def test_llcp_capped_lcps(sas):
    """SAS_ALGO_LLCP stores Llcp/Rlcp capped at 12 bits (SAS_LLCP_CAP = 4095).  Texts
    whose adjacent suffixes share far more than 4095 chars, with queries longer than
    the cap (exact matches, one-char mutations deep inside, text-end suffixes), take
    the capped branches; with and without the LDS / pivot-array top levels, every
    position equals the oracle's binary_search (sas/sa_search.rs:98-112)."""
    from sas_amd import _lib
    rng = np.random.default_rng(11)
    blk = rng.integers(0, 4, 6000, dtype=np.uint8)
    texts = {
        "all_A": np.zeros(20_000, np.uint8),
        "period_3": np.tile(np.array([0, 2, 1], np.uint8), 7000),
        "repeats": np.concatenate([blk, rng.integers(0, 4, 50, dtype=np.uint8), blk, blk[:5000], blk]),
    }
    for name, t in texts.items():
        n = len(t)
        idx = sas.SaNaive.build(t, verify=True, stree=False, sector=False, quad=True, prefix=False)
        assert idx.stats()["llcp_bytes"] == 16 * n
        sa = O.build_sa(t)
        qs = []
        for m in (1, 31, 33, 300, 4094, 4095, 4096, 4200, 6500):
            if m >= n:
                continue
            for o in rng.integers(0, n - m, 12):
                q = t[o:o + m].copy()
                qs.append(q)
                if m > 2:
                    for k in (m // 2, m - 1, min(m - 1, 4100)):
                        mq = q.copy()
                        mq[k] = (mq[k] + 1 + rng.integers(0, 3)) % 4
                        qs.append(mq)
        qs += [np.concatenate([t[n - k:], np.zeros(j, np.uint8)]) for k in (1, 4096, 5000) for j in (0, 3)]
        buf, qo, ql = pack(qs)
        expect = oracle_positions(t, sa, buf[:-64], qo, ql)
        for flags in (0, _lib.SAS_NO_LDS_TOP):
            for algo in ("plain", "llcp", "quad_llcp"):
                got, probes = idx.search_batch(buf, qo, ql, algo=algo, probes=True, flags=flags)
                assert np.array_equal(got, expect), (name, algo, flags, np.nonzero(got != expect)[0][:5])


def test_prefix_table(sas, sadef):
    """SAS_ALGO_PREFIX: the reference's prefix table (sas/sa_search.rs:59-95) for
    p = 1..16 chars, on fused and compact (u32 / 40-bit SA) quad leaves.  Random and
    repeat-rich texts give empty, single and very long key ranges and long gaps in
    the table (the workgroup-filled gap list); queries of every length 0..300,
    including m < p, positives, negatives and text-end suffixes, equal the oracle."""
    from sas_amd import _lib
    rng = np.random.default_rng(5)
    texts = {c["name"]: np.array(c["text"], np.uint8) for c in sadef["cases"]}
    texts["random_200k"] = sas.random_string(200_003, seed=77)
    texts["all_A"] = np.zeros(30_000, np.uint8)
    texts["period_5"] = np.tile(np.array([3, 1, 0, 2, 2], np.uint8), 8000)
    for name, t in texts.items():
        n = len(t)
        sa = O.build_sa(t)
        qs = [t[o:o + l] for o, l in zip(rng.integers(0, n, 400), rng.integers(0, 301, 400))]
        qs += [rng.integers(0, 4, l, dtype=np.uint8) for l in rng.integers(0, 40, 200)]
        qs += [t[n - k:] for k in (1, 2, 17, min(n, 40))] + [np.zeros(0, np.uint8), np.full(20, 3, np.uint8)]
        buf, qo, ql = pack(qs)
        expect = oracle_positions(t, sa, buf[:-64], qo, ql)
        for p, quad, sa40, inl in ((0, True, False, 0), (1, True, False, 0), (2, "compact", False, 0),
                                   (7, True, False, 0), (16, "compact", True, 0), (11, "compact", False, 0),
                                   (0, True, False, 1), (1, True, False, 1), (7, True, False, 1),
                                   (13, True, False, 1), (0, True, False, 2), (1, True, False, 2),
                                   (7, True, False, 2), (12, True, False, 2), (0, True, False, 4),
                                   (1, True, False, 4), (7, True, False, 4), (12, True, False, 4)):
            idx = sas.SaNaive.build(t, lcp=False, stree=False, sector=False, llcp=False, quad=quad, sa40=sa40,
                                    prefix=p if p else True, prefix_inline=inl)
            st = idx.stats()
            l4 = next(k for k in range(33) if 4 ** k >= n)  # ceil(log4 n)
            assert st["prefix_chars"] == (p if p else min(16, l4 + 1)), (name, p)
            assert st["prefix_bytes"] == (4 ** st["prefix_chars"] + 1) * (16 * inl if inl else 5 if sa40 else 4)
            got, probes = idx.search_batch(buf, qo, ql, algo="prefix", probes=True)
            assert np.array_equal(got, expect), (name, p, quad, sa40, inl, np.nonzero(got != expect)[0][:5])
            # the reference's own binary_search over SA + text, started from the table's range
            rng_probes = {}
            for base in ("plain", "lcp"):
                g2, rng_probes[base] = idx.search_batch(buf, qo, ql, algo=base, probes=True,
                                                        flags=_lib.SAS_PREFIX_RANGE)
                assert np.array_equal(g2, expect), (name, p, base, "range")
            assert np.array_equal(rng_probes["plain"], probes)  # same cnt as PREFIX
            if p == 7 and name == "random_200k":
                # cnt as the reference counts it (sas/sa_search.rs:86-112): 1 for the table
                # (p > 0), then one per binary-search iteration over [table[K], table[K+1])
                keys = np.array([int("".join(str(c) for c in t[x:x + 7]).ljust(7, "0"), 4) for x in sa])
                tb = bytes(t)
                for k, q in enumerate(qs[:300]):
                    K = int("".join(str(c) for c in q[:7]).ljust(7, "0"), 4)
                    lo, hi = np.searchsorted(keys, K, "left"), np.searchsorted(keys, K + 1, "left")
                    cnt, qq = 1, bytes(q)
                    while lo < hi:
                        mid = (lo + hi) // 2
                        cnt += 1
                        if tb[sa[mid]:sa[mid] + len(qq)] < qq:
                            lo = mid + 1
                        else:
                            hi = mid
                    assert (sa[lo] if lo < n else n) == got[k], k
                    assert probes[k] == cnt, (k, probes[k], cnt)
            del idx
    # built only with a quad tree, and refused without the table
    with pytest.raises(sas.SasError):
        sas.SaNaive.build(texts["random_200k"], quad=False, prefix=True)
    with pytest.raises(sas.SasError):  # inline entries need fused leaves
        sas.SaNaive.build(texts["random_200k"], quad="compact", prefix=True, prefix_inline=True)
    idx = sas.SaNaive.build(texts["random_200k"], prefix=False)
    with pytest.raises(sas.SasError):
        idx.search_batch(buf, qo, ql, algo="prefix")
    with pytest.raises(sas.SasError):
        idx.search_batch(buf, qo, ql, algo="plain", flags=_lib.SAS_PREFIX_RANGE)
    idx = sas.SaNaive.build(texts["random_200k"], prefix=True)
    with pytest.raises(sas.SasError):  # LLCP's entries belong to the intervals from [0, n)
        idx.search_batch(buf, qo, ql, algo="llcp", flags=_lib.SAS_PREFIX_RANGE)


def test_extract_substrings(sas):
    """sas_extract: substrings of the indexed text from its packed copy (what the c3
    bench cuts its queries from after dropping the byte text), 0 past the end."""
    import torch
    n = 100_003
    t = sas.random_string(n, seed=23)
    idx = sas.SaNaive.build(t, lcp=False, stree=False, sector=False, quad=False, llcp=False)
    rng = np.random.default_rng(4)
    pos = np.concatenate([rng.integers(0, n, 500), [0, n - 1, n - 5, n]]).astype(np.int64)
    lens = np.concatenate([rng.integers(0, 300, 500), [40, 1, 12, 3]]).astype(np.int32)
    off = np.zeros(len(pos), np.int64)
    off[1:] = np.cumsum(lens[:-1])
    out = torch.full((int(lens.sum()),), 9, dtype=torch.uint8, device="cuda")
    idx.extract(torch.from_numpy(pos).cuda(), torch.from_numpy(lens).cuda(), torch.from_numpy(off).cuda(), out)
    got = out.cpu().numpy()
    tp = np.concatenate([t, np.zeros(400, np.uint8)])
    for p_, l_, o_ in zip(pos, lens, off):
        assert np.array_equal(got[o_:o_ + l_], tp[p_:p_ + l_]), (p_, l_)


def test_packed_queries(sas):
    """sas_pack_queries / sas_search_packed: 2-bit packed fixed-length queries (first char
    high, as string_value<K> packs them, sas/util.rs:76-117) give the byte queries'
    positions, on rank and inline prefix tables, host and device pointers."""
    import torch
    n = 300_007
    t = sas.random_string(n, seed=52)
    sa = O.build_sa(t)
    rng = np.random.default_rng(8)
    for inl in (0, 2):
        idx = sas.SaNaive.build(t, stree=False, sector=False, llcp=False, lcp=False, prefix=True, prefix_inline=inl)
        for m in (1, 7, 16, 31, 32):
            offs = rng.integers(0, n - m, 3000)
            qb = np.concatenate([np.concatenate([t[o:o + m] for o in offs]),
                                 rng.integers(0, 4, 500 * m, dtype=np.uint8)])
            nq = len(qb) // m
            expect = oracle_positions(t, sa, qb, np.arange(nq, dtype=np.uint64) * m, np.full(nq, m, np.uint32))
            words = sas.SaNaive.pack_queries(torch.from_numpy(qb).cuda(), m)
            ref = np.array([int("".join(str(c) for c in qb[k * m:(k + 1) * m]).ljust(32, "0"), 4) for k in range(nq)],
                           np.uint64)
            assert np.array_equal(words.cpu().numpy().view(np.uint64), ref), m
            got = idx.search_packed(words, m).cpu().numpy().view(np.uint64)
            assert np.array_equal(got, expect), (inl, m)
            got_h, pr = idx.search_packed(ref, m, probes=True)
            assert np.array_equal(got_h, expect), (inl, m)
            _, pr_b = idx.search_fixed(qb, m, algo="prefix", probes=True)
            assert np.array_equal(pr, pr_b), (inl, m)
    with pytest.raises(sas.SasError):
        sas.SaNaive.pack_queries(torch.full((64,), 5, dtype=torch.uint8, device="cuda"), 32)
    with pytest.raises(sas.SasError):
        idx.search_packed(ref, 32, algo="quad")


def test_concurrent_calls_keep_their_error_flags(sas):
    """The index is immutable and may be searched from several threads at once
    (SearchIndex: Sync, sst/lib.rs:30): a call with invalid query codes
    fails, a concurrent valid call on the same index does not, and its answers hold."""
    from concurrent.futures import ThreadPoolExecutor
    n = 50_000
    t = sas.random_string(n, seed=41)
    idx = sas.SaNaive.build(t, stree=False, sector=False, llcp=False)
    sa = O.build_sa(t)
    rng = np.random.default_rng(6)
    qs = [t[o:o + 32] for o in rng.integers(0, n - 40, 4000)]
    buf, off, lens = pack(qs)
    expect = oracle_positions(t, sa, buf[:-64], off, lens)
    bad = buf.copy()
    bad[5] = 7

    def good_call(_):
        return idx.search_batch(buf, off, lens, algo="prefix")

    def bad_call(_):
        try:
            idx.search_batch(bad, off, lens, algo="prefix")
        except sas.SasError:
            return True
        return False

    with ThreadPoolExecutor(8) as ex:
        goods = [ex.submit(good_call, k) for k in range(24)]
        bads = [ex.submit(bad_call, k) for k in range(24)]
        for f in goods:
            assert np.array_equal(f.result(), expect)
        assert all(f.result() for f in bads)


def test_invalid_codes_rejected(sas):
    with pytest.raises(sas.SasError):
        sas.SaNaive.build(np.array([0, 1, 4, 2], np.uint8))
    idx = sas.SaNaive.build(np.array([0, 1, 2, 3] * 10, np.uint8))
    with pytest.raises(sas.SasError):
        idx.search([np.array([0, 1, 7], np.uint8)])
    with pytest.raises(sas.SasError):
        sas.SaNaive.build(np.zeros(0, np.uint8))


def test_reference_api_shapes(sas):
    t = sas.random_string(5000)
    idx = sas.SaNaive.build(t)
    sa = O.build_sa(t)
    tp = O.padded(t)
    cnt = sas.Counter()
    q = t[1000:1040]
    assert sas.binary_search(idx, q, cnt) == O.search_one(tp, len(t), sa, q)[0]
    assert cnt.value == O.search_one(tp, len(t), sa, q)[1]
    qs = [t[i:i + 35] for i in range(0, 4000, 97)]
    assert sas.binary_search_batch(idx, qs) == [O.search_one(tp, len(t), sa, x)[0] for x in qs]


def test_device_pointer_path(sas):
    import torch
    n, nq, m = 1 << 18, 4096, 32
    t = sas.random_string(n, device="cuda")
    ht = t.cpu().numpy()
    assert np.array_equal(ht, O.random_string(n))
    idx = sas.SaNaive.build(t, lcp=False, stree=True)
    off, _, _ = sas.random_queries(n, nq, len_lo=m, len_hi=m + 1)
    qb = torch.from_numpy(np.concatenate([ht[o:o + m] for o in off.astype(np.int64)])).cuda()
    host = idx.search_fixed(qb.cpu().numpy(), m, algo="plain")
    for algo in ALGOS:
        dev = idx.search_fixed(qb, m, algo=algo)
        torch.cuda.synchronize()
        assert np.array_equal(dev.cpu().numpy().astype(np.uint64), host), algo
    out = torch.empty(nq, dtype=torch.int64, device="cuda")
    kns, cns = idx.time_fixed(qb, m, nq, out, algo="stree", reps=3)
    assert kns > 0 and np.array_equal(out.cpu().numpy().astype(np.uint64), host)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_indexes_single_gpu(sas, world):
    """Sharded-text mode on one GPU: W shard indexes (global SA rank ranges),
    queries routed by sas_route, answered by their shard == the whole index."""
    from sas_amd.shard import shard_range
    n, nq, m = 200_003, 20_000, 24
    t = sas.random_string(n, seed=11)
    full = sas.SaNaive.build(t)
    sa = full.suffix_array()
    shards = [sas.SaNaive.build(t, sa=sa, rank_range=shard_range(n, world, g)) for g in range(world)]
    for g, s in enumerate(shards):
        lo, hi = shard_range(n, world, g)
        st = s.stats()
        assert st["rank_lo"] == lo and st["sa_entries"] == hi - lo
        assert st["next_pos"] == (sa[hi] if hi < n else n)
        assert np.array_equal(s.suffix_array(), sa[lo:hi])
    splitters = np.array([sa[shard_range(n, world, g)[0]] for g in range(1, world)], np.uint64)
    off, _, _ = sas.random_queries(n, nq, seed=3, len_lo=m, len_hi=m + 1)
    qb = np.concatenate([t[o:o + m] for o in off.astype(np.int64)])
    rng = np.random.default_rng(0)
    qb[: (nq // 4) * m] = rng.integers(0, 4, (nq // 4) * m, dtype=np.uint8)
    expect = full.search_fixed(qb, m, algo="plain")
    dest = shards[0].route(splitters, qb, m)
    assert dest.max() < world
    got = np.zeros(nq, np.uint64)
    for g in range(world):
        sel = np.nonzero(dest == g)[0]
        if len(sel) == 0:
            continue
        sub = qb.reshape(nq, m)[sel].reshape(-1)
        for algo in ALGOS:
            r = shards[g].search_fixed(sub, m, algo=algo)
            assert np.array_equal(r, expect[sel]), (world, g, algo)
        got[sel] = r
    assert np.array_equal(got, expect)


def test_wide_doubling_rounds(sas, sadef):
    """The n >= 2^31 builder path (two stable radix passes per doubling round),
    forced at small n, must give the same SA as the definition oracle."""
    from sas_amd import _lib
    for c in sadef["cases"]:
        t = np.array(c["text"], np.uint8)
        idx = sas.SaNaive.build(t, verify=True, flags=_lib.SAS_BUILD_WIDE)
        assert idx.suffix_array().tolist() == c["sa"], c["name"]
    rng = np.random.default_rng(9)
    blk = rng.integers(0, 4, 3000, dtype=np.uint8)
    for t in (np.zeros(70_000, np.uint8), np.concatenate([blk, blk, rng.integers(0, 4, 999, dtype=np.uint8), blk])):
        idx = sas.SaNaive.build(t, verify=True, flags=_lib.SAS_BUILD_WIDE)
        assert np.array_equal(idx.suffix_array(), O.build_sa(t))
        assert idx.stats()["sa_rounds"] > 0


def test_large_text_sampled(sas):
    """n > 2^31 (the wide builder path for real): GPU adjacency + permutation
    check (sas/sa_search.rs:36-38) and sampled positions vs the oracle."""
    import torch
    n = (1 << 31) + 12345
    t = sas.random_string(n, seed=123, device="cuda")
    idx = sas.SaNaive.build(t, lcp=False, stree=True, llcp=True, verify=True)
    ht = t.cpu().numpy()
    del t
    torch.cuda.empty_cache()
    sa = idx.suffix_array()
    nq, m = 4096, 40
    off, _, _ = sas.random_queries(n, nq, seed=5, len_lo=m, len_hi=m + 1)
    qb = np.concatenate([ht[o:o + m] for o in off.astype(np.int64)])
    rng = np.random.default_rng(1)
    qb[: 512 * m] = rng.integers(0, 4, 512 * m, dtype=np.uint8)
    expect = oracle_positions(ht, sa, qb, np.arange(nq, dtype=np.uint64) * m, np.full(nq, m, np.uint32))
    for algo in ALGOS:
        assert np.array_equal(idx.search_fixed(qb, m, algo=algo), expect), algo


def test_ragged_unaligned_device_queries(sas):
    """Ragged queries at odd byte offsets in an exactly-sized device buffer (no
    padding after the last query): the aligned-block realignment must read only
    blocks that hold query bytes, and answers must match the host path."""
    import torch
    n = 300_007
    t = sas.random_string(n, seed=21)
    idx = sas.SaNaive.build(t)
    rng = np.random.default_rng(4)
    lens = rng.integers(0, 300, 5000).astype(np.uint32)
    starts = rng.integers(0, n - 300, 5000)
    qs = [t[s:s + l] for s, l in zip(starts, lens)]
    buf = np.concatenate([np.array([1, 2, 3], np.uint8)] + qs)  # odd base offset
    off = (np.concatenate([[0], np.cumsum(lens[:-1])]) + 3).astype(np.uint64)
    expect = idx.search_batch(np.concatenate([buf, np.zeros(64, np.uint8)]), off, lens, algo="plain")
    dbuf = torch.from_numpy(buf).cuda()
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    dlen = torch.from_numpy(lens.view(np.int32)).cuda()
    for algo in ALGOS:
        got = idx.search_batch(dbuf, doff, dlen, algo=algo)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy().astype(np.uint64), expect), algo
    sa = idx.suffix_array()
    assert np.array_equal(expect, oracle_positions(t, sa, buf, off, lens))


def test_occurrence_ranges(sas, sadef):
    """sas_search_range (Search::search_prefix, sas/util.rs:36-40): SA[lo:hi] is
    exactly the set of occurrences, on the definition fixtures, random texts with
    mixed queries (vs the oracle) and long runs."""
    for c in sadef["cases"]:
        t = np.array(c["text"], np.uint8)
        idx = sas.SaNaive.build(t)
        buf, off, lens = pack([q["q"] for q in c["queries"]])
        lo, hi = idx.search_range(buf, off, lens)
        sa = np.array(c["sa"], np.uint32)
        tl = c["text"]
        for k, qd in enumerate(c["queries"]):
            q = qd["q"]
            assert lo[k] == qd["rank"], (c["name"], q)
            occ = sorted(i for i in range(len(tl)) if tl[i:i + len(q)] == q) if len(q) <= len(tl) else []
            assert sorted(sa[lo[k]:hi[k]].tolist()) == occ, (c["name"], q)
    rng = np.random.default_rng(8)
    for t in (sas.random_string(1 << 20, seed=77), np.zeros(50_000, np.uint8),
              np.tile(rng.integers(0, 4, 13, dtype=np.uint8), 9000)):
        n = len(t)
        idx = sas.SaNaive.build(t)
        sa = idx.suffix_array()
        tp = O.padded(t)
        qs = [t[o:o + l] for o, l in zip(rng.integers(0, n - 300, 3000), rng.integers(0, 300, 3000))]
        qs += [rng.integers(0, 4, rng.integers(1, 12), dtype=np.uint8) for _ in range(1000)]
        buf, off, lens = pack(qs)
        lo, hi = idx.search_range(buf, off, lens)
        for k, q in enumerate(qs):
            assert (lo[k], hi[k]) == O.prefix_range(tp, n, sa, q), (n, k, len(q))
    t = np.zeros(1000, np.uint8)
    idx = sas.SaNaive.build(t)
    assert sorted(idx.search_prefix(np.zeros(10, np.uint8)).tolist()) == list(range(991))


def test_occurrence_ranges_both_trees(sas, sadef):
    """sas_search_range runs on the prefix table when it is built (k_sa_prefix_range, any
    entry format), on the quad tree otherwise (k_sa_quad_range) and on the sector tree
    without one (k_sa_sector_range): all give identical ranges, including
    above-every-suffix, empty and long queries, and a quad-only index searches."""
    from sas_amd import _lib
    rng = np.random.default_rng(21)
    cases = [np.array(c["text"], np.uint8) for c in sadef["cases"]]
    cases += [sas.random_string(300_000, seed=5), np.zeros(20_000, np.uint8),
              np.tile(rng.integers(0, 4, 5, dtype=np.uint8), 4000)]
    for t in cases:
        n = len(t)
        q_only = sas.SaNaive.build(t, lcp=False, stree=False, sector=False, quad=True)
        s_only = sas.SaNaive.build(t, lcp=False, stree=False, sector=True, quad=False)
        qs = [t[o:o + l] for o, l in zip(rng.integers(0, max(1, n - 1), 400), rng.integers(0, 300, 400))]
        qs += [np.full(l, 3, np.uint8) for l in (1, 16, 31, 32, 33, 64, 200)]  # above every suffix
        qs += [rng.integers(0, 4, l, dtype=np.uint8) for l in rng.integers(0, 70, 200)]
        buf, off, lens = pack(qs)
        lq, hq = q_only.search_range(buf, off, lens)  # prefix table (built with the quad tree)
        ls, hs = s_only.search_range(buf, off, lens)
        assert np.array_equal(lq, ls) and np.array_equal(hq, hs), n
        lt, ht = q_only.search_range(buf, off, lens, flags=_lib.SAS_NO_PREFIX_TABLE)  # quad descents
        assert np.array_equal(lq, lt) and np.array_equal(hq, ht), n
        for inl in (1, 2):
            qi = sas.SaNaive.build(t, lcp=False, stree=False, sector=False, llcp=False, quad=True, prefix=True,
                                   prefix_inline=inl)
            li, hi = qi.search_range(buf, off, lens)
            assert np.array_equal(lq, li) and np.array_equal(hq, hi), (n, inl)
        assert np.array_equal(q_only.search_batch(buf, off, lens, algo="quad"),
                              s_only.search_batch(buf, off, lens, algo="sector")), n


def test_quad_relative_nodes(sas, sadef):
    """Quad inner nodes: prefix-relative (SAS_BUILD_QUAD_REL, 31-ary: a node's shared
    d-char prefix + 30 16-bit separators over the next 8 chars) and absolute
    (SAS_BUILD_QUAD_ABS, 17-ary 16-char separators) must both give the oracle's
    positions and identical ranges; the automatic choice is absolute at these sizes.
    Queries mutated at chars 0..24 land between separators at every depth and exercise
    the below/above-prefix cases; leaf counts of 31^k + 1 leave a one-child last node
    per layer (the clamp), and a near-periodic text pins d at its 13-char cap."""
    rng = np.random.default_rng(31)
    per = np.tile(rng.integers(0, 4, 16, dtype=np.uint8), 4000)
    per[rng.integers(0, len(per), 300)] = rng.integers(0, 4, 300, dtype=np.uint8)
    texts = [sas.random_string(1_000_003, seed=12), sas.random_string(4 * 31 ** 3 + 1, seed=13),
             sas.random_string(4 * 31 ** 2 + 3, seed=14), np.zeros(50_000, np.uint8), per,
             np.tile(rng.integers(0, 4, 13, dtype=np.uint8), 7000)]
    texts += [np.array(c["text"], np.uint8) for c in sadef["cases"]]
    assert sas.SaNaive.build(texts[0], lcp=False, stree=False, sector=False).stats()["quad_fan"] == 17
    for t in texts:
        n = len(t)
        for leaves in ("", "compact-"):
            rel = sas.SaNaive.build(t, lcp=False, stree=False, sector=False, quad=leaves + "rel")
            ab = sas.SaNaive.build(t, lcp=False, stree=False, sector=False, quad=leaves + "abs")
            assert rel.stats()["quad_fan"] == 31 and ab.stats()["quad_fan"] == 17
            quad = leaves or "fused"
            sa = rel.suffix_array()
            qs = []
            for o, l in zip(rng.integers(0, max(1, n - 40), 1500), rng.integers(1, 40, 1500)):
                q = t[o:o + l].copy()
                if len(q):
                    j = rng.integers(0, len(q))
                    q[j] = (q[j] + rng.integers(1, 4)) % 4
                qs.append(q)
            qs += [t[o:o + l] for o, l in zip(rng.integers(0, max(1, n - 300), 800), rng.integers(0, 300, 800))]
            qs += [np.full(l, 3, np.uint8) for l in (1, 8, 13, 31, 32, 33, 200)] + [np.zeros(0, np.uint8)]
            qs += [t[n - k:] for k in (1, 5, 32, 40) if k <= n]
            buf, off, lens = pack(qs)
            expect = oracle_positions(t, sa, buf, off, lens)
            for idx in (rel, ab):
                assert np.array_equal(idx.search_batch(buf, off, lens, algo="quad"), expect), (n, quad)
            if n >= 64:
                q32 = [t[o:o + 32].copy() for o in rng.integers(0, n - 32, 1500)]
                for q in q32[::2]:
                    j = rng.integers(0, 32)
                    q[j] = (q[j] + 1) % 4
                q32 += [np.full(32, 3, np.uint8)]
                b32 = np.concatenate(q32)
                e32 = oracle_positions(t, sa, b32, np.arange(len(q32), dtype=np.uint64) * 32,
                                       np.full(len(q32), 32, np.uint32))
                assert np.array_equal(rel.search_fixed(b32, 32, algo="quad"), e32), (n, quad)
            lr, hr = rel.search_range(buf, off, lens)
            la, ha = ab.search_range(buf, off, lens)
            assert np.array_equal(lr, la) and np.array_equal(hr, ha), (n, quad)


def test_compact_quad_leaves(sas, sadef):
    """SAS_BUILD_QUAD_COMPACT: key-only quad leaves (8 per 64-B leaf, SA values from the
    SA array), u32 and 40-bit SA.  QUAD (cooperative m <= 32 kernel and the 4x kernel
    for longer queries), INLINE and occurrence ranges equal the oracle / the fused
    index on the definition fixtures, random, all-zero, periodic and repeat texts."""
    rng = np.random.default_rng(44)
    for c in sadef["cases"]:
        t = np.array(c["text"], np.uint8)
        buf, off, lens = pack([q["q"] for q in c["queries"]])
        expect = np.array([q["pos"] for q in c["queries"]], np.uint64)
        for sa40 in (False, True):
            idx = sas.SaNaive.build(t, lcp=False, stree=False, sector=False, quad="compact", sa40=sa40)
            assert idx.stats()["quad_entry_bytes"] == 8
            for algo in ("quad", "inline"):
                assert np.array_equal(idx.search_batch(buf, off, lens, algo=algo), expect), (c["name"], sa40, algo)
            lo, _ = idx.search_range(buf, off, lens)
            assert lo.tolist() == [q["rank"] for q in c["queries"]], c["name"]
    blk = rng.integers(0, 4, 3000, dtype=np.uint8)
    texts = [sas.random_string(2_000_003, seed=9), np.zeros(40_000, np.uint8),
             np.tile(rng.integers(0, 4, 7, dtype=np.uint8), 12_000),
             np.concatenate([blk, blk, rng.integers(0, 4, 999, dtype=np.uint8), blk, blk[:1777]])]
    for t in texts:
        n = len(t)
        fused = sas.SaNaive.build(t, lcp=False, stree=False, sector=False, quad=True)
        sa = fused.suffix_array()
        assert fused.stats()["quad_entry_bytes"] == 16
        qs = [t[o:o + l] for o, l in zip(rng.integers(0, n - 300, 3000), rng.integers(1, 300, 3000))]
        qs += [rng.integers(0, 4, rng.integers(0, 70), dtype=np.uint8) for _ in range(800)]
        qs += [np.full(l, 3, np.uint8) for l in (1, 31, 32, 33, 200)] + [t[n - k:] for k in (1, 5, 32, 40)]
        buf, off, lens = pack(qs)
        expect = oracle_positions(t, sa, buf, off, lens)
        q32 = [t[o:o + 32] for o in rng.integers(0, n - 32, 3000)] + [np.full(32, 3, np.uint8)]
        b32 = np.concatenate(q32)
        e32 = oracle_positions(t, sa, b32, np.arange(len(q32), dtype=np.uint64) * 32,
                               np.full(len(q32), 32, np.uint32))
        flo, fhi = fused.search_range(buf, off, lens)
        for sa40 in (False, True):
            idx = sas.SaNaive.build(t, lcp=False, stree=False, sector=False, quad="compact", sa40=sa40)
            st = idx.stats()
            assert st["quad_bytes"] < fused.stats()["quad_bytes"] * 0.6
            for algo in ("quad", "inline"):
                assert np.array_equal(idx.search_batch(buf, off, lens, algo=algo), expect), (n, sa40, algo)
                assert np.array_equal(idx.search_fixed(b32, 32, algo=algo), e32), (n, sa40, algo)
            lo, hi = idx.search_range(buf, off, lens)
            assert np.array_equal(lo, flo) and np.array_equal(hi, fhi), (n, sa40)


def test_kmer_keys_match_reference_loop(sas):
    """sst/bin/bench.rs:58-76 (--human keys), restated as the reference's loop."""
    t = sas.random_string(5000, seed=2)
    for k, limit in ((16, 5000), (16, 1000), (11, 4990), (16, 10)):
        key, vals = 0, []
        for i in range(k - 1):
            key = key << 2 | int(t[i])
        for i in range(k - 1, min(len(t), limit + k - 1)):
            key = (key << 2 | int(t[i])) & ((1 << (2 * k)) - 1)
            vals.append(key & 0x7FFFFFFF)
        vals[0] = 0x7FFFFFFF
        assert sas.kmer_keys(t, k, limit).tolist() == vals, (k, limit)
    keys = np.sort(sas.kmer_keys(t))
    idx = sas.STree16.new(keys)  # the S-tree the reference builds over them
    qs = np.sort(keys)[::7]
    assert np.array_equal(idx.query(qs), O.SortedVec(keys).query(qs))


def test_sa40_matches_u32_path(sas, sadef):
    """Packed 40-bit SA + bucketed builder (the n >= 2^32 path), forced at small
    n: the SA is bit-identical to the oracle's, every algorithm returns the same
    positions as the u32 index, occurrence ranges and shards agree."""
    for c in sadef["cases"]:
        t = np.array(c["text"], np.uint8)
        idx = sas.SaNaive.build(t, verify=True, sa40=True)
        assert idx.stats()["sa_width"] == 5
        assert idx.suffix_array().tolist() == c["sa"], c["name"]
        buf, off, lens = pack([q["q"] for q in c["queries"]])
        expect = np.array([q["pos"] for q in c["queries"]], np.uint64)
        for algo in ALGOS:
            assert np.array_equal(idx.search_batch(buf, off, lens, algo=algo), expect), (c["name"], algo)
    rng = np.random.default_rng(12)
    blk = rng.integers(0, 4, 3000, dtype=np.uint8)
    texts = [sas.random_string(3_000_017, seed=4), np.zeros(70_000, np.uint8),
             np.concatenate([blk, blk, rng.integers(0, 4, 999, dtype=np.uint8), blk]),
             np.tile(rng.integers(0, 4, 7, dtype=np.uint8), 20_000)]
    for t in texts:
        n = len(t)
        a = sas.SaNaive.build(t, verify=True)
        b = sas.SaNaive.build(t, verify=True, sa40=True)
        sa = a.suffix_array()
        assert np.array_equal(b.suffix_array(), sa.astype(np.uint64)), n
        assert np.array_equal(b.lcp_array(), a.lcp_array())
        qs = [t[o:o + l] for o, l in zip(rng.integers(0, n - 300, 2000), rng.integers(1, 300, 2000))]
        qs += [rng.integers(0, 4, rng.integers(1, 40), dtype=np.uint8) for _ in range(500)]
        buf, off, lens = pack(qs)
        expect = oracle_positions(t, sa, buf, off, lens)
        for algo in ALGOS:
            assert np.array_equal(b.search_batch(buf, off, lens, algo=algo), expect), (n, algo)
        lo, hi = b.search_range(buf, off, lens)
        lo2, hi2 = a.search_range(buf, off, lens)
        assert np.array_equal(lo, lo2) and np.array_equal(hi, hi2)
        # caller-supplied u64 SA, and 40-bit shards
        c64 = sas.SaNaive.build(t, sa=sa.astype(np.uint64), verify=True, lcp=False)
        assert c64.stats()["sa_width"] == 4 and np.array_equal(c64.suffix_array(), sa)
        from sas_amd.shard import shard_range
        for g in range(2):
            lo_r, hi_r = shard_range(n, 2, g)
            s = sas.SaNaive.build(t, sa=sa, rank_range=(lo_r, hi_r), sa40=True)
            assert np.array_equal(s.suffix_array(), sa[lo_r:hi_r].astype(np.uint64))
            assert s.stats()["next_pos"] == (sa[hi_r] if hi_r < n else n)


def test_sa_beyond_u32(sas):
    """n > 2^32 (past the reference's u32 SA, sas/sa_search.rs:35): the 40-bit
    builder for real.  The SA is checked on the GPU (adjacency as
    sas/sa_search.rs:36-38 + permutation); every answer is then proven to be the
    exact lower bound on the host text: SA[lo-1] < q <= SA[lo], pos = SA[lo].  The
    compact-leaf, LLCP, 40-bit prefix-table and bucket-line indexes of the same text
    return the same positions and ranges."""
    import torch
    n = (1 << 32) + 12345
    t = sas.random_string(n, seed=321, device="cuda")
    idx = sas.SaNaive.build(t, lcp=False, stree=True, verify=True, llcp=False)  # LLCP: the second index below
    st = idx.stats()
    assert st["sa_width"] == 5 and st["n"] == n
    algos = [a for a in ALGOS if a not in ("llcp", "prefix", "interp", "stree_llcp", "quad_llcp")]  # prefix: u32 ranks; interp: n < 2^32
    ht = t.cpu().numpy()
    del t
    torch.cuda.empty_cache()
    rng = np.random.default_rng(2)
    nq = 3000
    offs = np.concatenate([rng.integers(0, n - 300, nq - 600), rng.integers((1 << 32) - 100, n - 300, 100)])
    qs = [ht[o:o + l] for o, l in zip(offs, rng.integers(8, 257, len(offs)))]
    qs += [rng.integers(0, 4, rng.integers(1, 30), dtype=np.uint8) for _ in range(500)]
    buf, off, lens = pack(qs)
    lo, hi = idx.search_range(buf, off, lens)
    got = {algo: idx.search_batch(buf, off, lens, algo=algo) for algo in algos}
    big = 0
    for k, q in enumerate(qs):
        qb = bytes(q)
        r = int(lo[k])
        pair = idx.suffix_array(count=2 if r > 0 else 1, start=r - 1 if r > 0 else 0)
        cur = int(pair[-1]) if r < n else n
        prev = int(pair[0]) if r > 0 else None
        if r < n:
            assert bytes(ht[cur:cur + len(q)]) >= qb, k
        if prev is not None:
            assert bytes(ht[prev:prev + len(q)]) < qb, k
        for algo in algos:
            assert int(got[algo][k]) == cur, (k, algo)
        big += cur >= (1 << 32)
        if k < 600:
            occ_hi = int(hi[k])
            if occ_hi > r:
                last = int(idx.suffix_array(count=1, start=occ_hi - 1)[0])
                assert bytes(ht[last:last + len(q)]) == qb
    assert big > 0  # positions above 2^32 were returned
    # compact quad leaves at the same n: SA values (above 2^32) come from the 40-bit array;
    # the LLCP entries carry 40-bit SA values too
    del idx
    torch.cuda.empty_cache()
    tc = torch.from_numpy(ht).cuda()
    cidx = sas.SaNaive.build(tc, lcp=False, stree=False, sector=False, quad="compact", prefix=16, llcp=True)
    del tc
    assert cidx.stats()["quad_entry_bytes"] == 8 and cidx.stats()["llcp_bytes"] == 16 * n
    assert cidx.stats()["prefix_bytes"] == (4 ** 16 + 1) * 5  # 40-bit ranks beside the 40-bit SA
    for algo in ("quad", "inline", "llcp", "prefix"):
        assert np.array_equal(cidx.search_batch(buf, off, lens, algo=algo), got["plain"]), algo
    clo, chi = cidx.search_range(buf, off, lens)
    assert np.array_equal(clo, lo) and np.array_equal(chi, hi)
    # bucket lines above 2^32 chars: 33-bit SA fields and 15-bit tags (an odd tag: the tie's
    # text compare starts at char p + 7); p = 14, ~16 suffixes a line
    cidx.free()
    torch.cuda.empty_cache()
    lidx = sas.SaNaive.build(ht, lcp=False, tagged=14, tag_lines=True)
    lst = lidx.stats()
    assert lst["tag_line_tag_bits"] == 15 and lst["tag_line_slots"] == 20 and lst["tag_chars"] == 14
    assert np.array_equal(lidx.search_batch(buf, off, lens, algo="tagged"), got["plain"])
    llo, lhi = lidx.search_range(buf, off, lens)
    assert np.array_equal(llo, lo) and np.array_equal(lhi, hi)
    for k in range(0, len(qs), 211):
        r = int(lo[k])
        if r < n:
            assert int(lidx.suffix_array(count=1, start=r)[0]) == int(got["plain"][k]), k


def test_llcp_tails_beyond_u32(sas):
    """The LCP-skipping tails with 64-bit ranks (n > 2^32: k_sa_quad_llcp<.., R32 = false>, the
    40-bit LLCP entries of STREE_LLCP and LLCP): 64 copies of a 400-char block that starts with
    20 'T's are planted in a 2^32 + 12345-char random text, so the copies' first suffixes sort
    at ranks above 2^32 in runs of 64 equal 32-char keys, each copy followed by different random
    text.  Queries of 33..256 chars from the copies' first 9 offsets (with one char changed past
    char 32 too), from positions above 2^32 and the text's last suffixes: QUAD_LLCP (on
    the absolute quad layout, which it needs), STREE_LLCP and LLCP equal PLAIN, and every PLAIN
    answer is proven the exact lower bound on the host text (sas/sa_search.rs:98-112)."""
    import torch
    n = (1 << 32) + 12345
    t = sas.random_string(n, seed=987, device="cuda")
    rng = np.random.default_rng(8)
    blk = torch.from_numpy(np.concatenate([np.full(20, 3, np.uint8), rng.integers(0, 4, 380, dtype=np.uint8)])).cuda()
    starts = np.sort(rng.choice(np.arange(1 << 20, n - 1000, 4096, dtype=np.int64), 64, replace=False))
    for s in starts:
        t[int(s):int(s) + 400] = blk
    ht = t.cpu().numpy()
    idx = sas.SaNaive.build(t, lcp=False, stree=True, sector=False, quad="abs", llcp=True, prefix=False)
    del t
    torch.cuda.empty_cache()
    st = idx.stats()
    assert st["sa_width"] == 5 and st["quad_fan"] == 17 and st["llcp_bytes"] == 16 * n
    qs = []
    for s in starts[:48]:
        for m in (33, 48, 64, 100, 200, 256):
            # >= 12 leading 'T's: among the text's top ~10^3 suffixes, ranks above 2^32
            o = int(s) + int(rng.integers(0, 9))
            q = ht[o:o + m].copy()
            qs.append(q)
            mq = q.copy()
            k = int(rng.integers(32, m))
            mq[k] = (mq[k] + 1 + rng.integers(0, 3)) % 4
            qs.append(mq)
    hi_offs = rng.integers((1 << 32) - 100, n - 300, 200)
    qs += [ht[o:o + m] for o, m in zip(hi_offs, rng.integers(33, 257, 200))]
    qs += [np.concatenate([ht[n - k:], np.zeros(j, np.uint8)]) for k in (20, 40, 300) for j in (0, 30)]
    buf, off, lens = pack(qs)
    plain = idx.search_batch(buf, off, lens, algo="plain")
    for algo in ("quad_llcp", "stree_llcp", "llcp"):
        got = idx.search_batch(buf, off, lens, algo=algo)
        bad = np.nonzero(got != plain)[0]
        assert len(bad) == 0, (algo, bad[:5])
    lo, _ = idx.search_range(buf, off, lens)
    above = 0
    for k, q in enumerate(qs):
        qb = bytes(q)
        r = int(lo[k])
        pair = idx.suffix_array(count=2 if r > 0 else 1, start=r - 1 if r > 0 else 0)
        cur = int(pair[-1]) if r < n else n
        assert int(plain[k]) == cur, k
        if r < n:
            assert bytes(ht[cur:cur + len(q)]) >= qb, k
        if r > 0:
            assert bytes(ht[int(pair[0]):int(pair[0]) + len(q)]) < qb, k
        above += r >= (1 << 32)
    assert above >= 48 * 12  # the planted copies' queries were answered at ranks above 2^32
    idx.free()


def test_fasta_genome_like_end_to_end(sas, tmp_path):
    """read_fasta_file (sas/util.rs:144-169) -> GPU SA -> every algorithm vs the oracle,
    on a genome-shaped FASTA: several records, soft-masked (lowercase) runs, long N
    stretches (-> code 0, so long runs of equal keys), tandem and interspersed repeats."""
    rng = np.random.default_rng(17)
    alpha = np.array(list("ACGT"))
    unit = "".join(alpha[rng.integers(0, 4, 300)])
    recs = []
    for r in range(4):
        parts = []
        for _ in range(30):
            kind = rng.integers(0, 4)
            if kind == 0:
                parts.append("".join(alpha[rng.integers(0, 4, rng.integers(500, 3000))]))
            elif kind == 1:
                parts.append("N" * int(rng.integers(50, 2000)))
            elif kind == 2:
                parts.append(unit * int(rng.integers(1, 6)))
            else:
                parts.append("".join(alpha[rng.integers(0, 4, rng.integers(100, 800))]).lower())
        seq = "".join(parts)
        recs.append(f">chr{r} synthetic\n" + "\n".join(seq[i:i + 60] for i in range(0, len(seq), 60)))
    path = tmp_path / "genome.fa"
    path.write_text("\n".join(recs) + "\n")
    t = sas.read_fasta_file(str(path))
    n = len(t)
    sa_ref = O.build_sa(t)
    idx = sas.SaNaive.build(t, verify=True)
    assert np.array_equal(idx.suffix_array(), sa_ref)
    qs = [t[o:o + l] for o, l in zip(rng.integers(0, n - 400, 3000), rng.integers(1, 400, 3000))]
    qs += [np.zeros(l, np.uint8) for l in (5, 40, 100, 1999, 2500)]  # inside / beyond the N runs
    buf, off, lens = pack(qs)
    expect = oracle_positions(t, sa_ref, buf, off, lens)
    for algo in ALGOS:
        assert np.array_equal(idx.search_batch(buf, off, lens, algo=algo), expect), algo
    lo, hi = idx.search_range(buf, off, lens)
    tp = O.padded(t)
    for k in range(0, len(qs), 7):
        assert (lo[k], hi[k]) == O.prefix_range(tp, n, sa_ref, qs[k])


@pytest.mark.parametrize("parts", [1, 2, 3, 5])
def test_part_builds_concatenate_to_full_sa(sas, parts):
    """sas_build_part: each part builds only its own SA rank range (no whole-SA
    step).  The parts' SAs concatenate to the oracle's SA, the ranges are
    contiguous, next_pos = SA[rank_hi], and routed lookups on the parts equal the
    whole index on mixed queries (sharded-text mode)."""
    rng = np.random.default_rng(parts)
    blk = rng.integers(0, 4, 700, dtype=np.uint8)
    texts = [sas.random_string(1_000_003, seed=9),
             np.concatenate([blk, rng.integers(0, 4, 5000, dtype=np.uint8), blk, blk,
                             rng.integers(0, 4, 3000, dtype=np.uint8), np.zeros(900, np.uint8), blk]),
             np.tile(rng.integers(0, 4, 7, dtype=np.uint8), 3000)]
    if parts == 1:
        texts.append(np.zeros(5000, np.uint8))
    for t in texts:
        n = len(t)
        sa_ref = O.build_sa(t)
        idxs = [sas.SaNaive.build_part(t, g, parts, verify=True) for g in range(parts)]
        st = [ix.stats() for ix in idxs]
        assert st[0]["rank_lo"] == 0 and sum(s["sa_entries"] for s in st) == n
        for g in range(parts):
            lo, cnt = st[g]["rank_lo"], st[g]["sa_entries"]
            assert st[g]["sa_width"] == 5
            if g + 1 < parts:
                assert st[g + 1]["rank_lo"] == lo + cnt
            assert np.array_equal(idxs[g].suffix_array(), sa_ref[lo:lo + cnt].astype(np.uint64)), (n, g)
            assert st[g]["next_pos"] == (sa_ref[lo + cnt] if lo + cnt < n else n)
        full = sas.SaNaive.build(t)
        m = 24
        offs = rng.integers(0, n - m, 3000)
        qb = np.concatenate([t[o:o + m] for o in offs] + [rng.integers(0, 4, 1000 * m, dtype=np.uint8)])
        nq = len(qb) // m
        expect = full.search_fixed(qb, m, algo="plain")
        splitters = np.array([idxs[g].suffix_array(1)[0] for g in range(1, parts)], np.uint64)
        dest = idxs[0].route(splitters, qb, m) if parts > 1 else np.zeros(nq, np.uint32)
        got = np.zeros(nq, np.uint64)
        for g in range(parts):
            sel = np.nonzero(dest == g)[0]
            if len(sel) == 0:
                continue
            sub = qb.reshape(nq, m)[sel].reshape(-1)
            for algo in ("quad", "plain", "stree"):
                assert np.array_equal(idxs[g].search_fixed(sub, m, algo=algo), expect[sel]), (n, g, algo)
            got[sel] = idxs[g].search_fixed(sub, m, algo="quad")
        assert np.array_equal(got, expect)


def test_part_builds_at_scale(sas):
    """n = 2^28 + 5, 3 parts: every part's SA equals the matching slice of the
    whole-SA builder's output; the ranges tile [0, n); next_pos links the parts."""
    n = (1 << 28) + 5
    t = sas.random_string(n, seed=44, device="cuda")
    full = sas.SaNaive.build(t, lcp=False, stree=False, sector=False, quad=False)
    sa = full.suffix_array()
    full.free()
    lo_expect = 0
    for g in range(3):
        ix = sas.SaNaive.build_part(t, g, 3, lcp=False, stree=False, sector=False, quad=True, verify=True)
        st = ix.stats()
        lo, cnt = st["rank_lo"], st["sa_entries"]
        assert lo == lo_expect and cnt > n // 4
        assert np.array_equal(ix.suffix_array(), sa[lo:lo + cnt].astype(np.uint64)), g
        assert st["next_pos"] == (int(sa[lo + cnt]) if lo + cnt < n else n)
        lo_expect = lo + cnt
        ix.free()
    assert lo_expect == n


def test_probe_counts_match_reference_counter(sas):
    """out_probes of PLAIN / LCP / LLCP = the reference's `cnt` of binary_search
    (sas/sa_search.rs:104: one per loop iteration while l < r), query by query,
    on the oracle's restatement; the Counter mirror sums them."""
    n = 200_003
    t = sas.random_string(n, seed=19)
    idx = sas.SaNaive.build(t)
    sa = idx.suffix_array()
    tp = O.padded(t)
    rng = np.random.default_rng(3)
    qs = [t[o:o + l] for o, l in zip(rng.integers(0, n - 100, 300), rng.integers(1, 80, 300))]
    qs += [rng.integers(0, 4, l, dtype=np.uint8) for l in rng.integers(1, 30, 200)]
    qs += [np.full(40, 3, np.uint8), np.zeros(0, np.uint8), t[n - 5:]]
    buf, off, lens = pack(qs)
    expect = [O.search_one(tp, n, sa, np.asarray(q, np.uint8), "binary_search") for q in qs]
    for algo in ("plain", "lcp", "llcp"):
        pos, probes = idx.search_batch(buf, off, lens, algo=algo, probes=True)
        assert pos.tolist() == [e[0] for e in expect], algo
        assert probes.tolist() == [e[1] for e in expect], algo
    cnt = sas.Counter()
    for q, e in zip(qs[:50], expect[:50]):
        assert sas.binary_search(idx, q, cnt) == e[0]
    assert cnt.value == sum(e[1] for e in expect[:50])


def test_route_pack(sas):
    """sas_route_pack: counts = histogram of sas_route's shards, slots are a
    permutation, every query's bytes sit at its slot inside its shard's bucket."""
    import torch
    n, m, W = 300_007, 24, 5
    t = sas.random_string(n, seed=61)
    idxs = [sas.SaNaive.build_part(t, g, W, lcp=False, stree=False, sector=False) for g in range(W)]
    splitters = torch.tensor([int(ix.suffix_array(1)[0]) for ix in idxs[1:]], dtype=torch.int64).cuda()
    rng = np.random.default_rng(2)
    offs = rng.integers(0, n - m, 20_000)
    qb = np.concatenate([t[o:o + m] for o in offs] + [rng.integers(0, 4, 5000 * m, dtype=np.uint8)])
    nq = len(qb) // m
    dq = torch.from_numpy(qb).cuda()
    dest = idxs[0].route(splitters, dq, m).cpu().numpy()
    counts, send, slot = idxs[0].route_pack(splitters, dq, m)
    counts, send, slot = counts.cpu().numpy(), send.cpu().numpy(), slot.cpu().numpy()
    assert counts.tolist() == np.bincount(dest, minlength=W).tolist()
    assert np.array_equal(np.sort(slot), np.arange(nq))
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    assert ((slot >= starts[dest]) & (slot < starts[dest] + counts[dest])).all()
    assert np.array_equal(send.reshape(nq, m)[slot], qb.reshape(nq, m))


def test_full_size_algorithms_agree_and_are_lower_bounds(sas):
    """BASELINE size (n = 2^30, 10^6 mixed queries: positive len 32 as in the bench,
    random negatives, other lengths), index as the bench builds it (p = 16 two-suffix
    inline prefix table): all algorithms return identical positions; a
    sample is proven exact on the host text (SA[lo-1] < q <= SA[lo], pos = SA[lo])."""
    import torch
    n = 1 << 30
    t = sas.random_string(n, seed=31415, device="cuda")
    idx = sas.SaNaive.build(t, prefix=16, prefix_inline=2)  # the bench's two-suffix inline table
    ht = t.cpu().numpy()
    rng = np.random.default_rng(30)
    offs = rng.integers(0, n - 200, 700_000)
    qs = [ht[o:o + 32] for o in offs[:500_000]]
    qs += [ht[o:o + l] for o, l in zip(offs[500_000:], rng.integers(1, 160, 200_000))]
    qs += [rng.integers(0, 4, l, dtype=np.uint8) for l in rng.integers(1, 40, 300_000)]
    buf, off, lens = pack(qs)
    dbuf = torch.from_numpy(buf).cuda()
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    dlen = torch.from_numpy(lens.view(np.int32)).cuda()
    res = {}
    for algo in ALGOS:
        res[algo] = idx.search_batch(dbuf, doff, dlen, algo=algo).cpu().numpy()
    for algo in ALGOS:
        assert np.array_equal(res[algo], res["plain"]), algo
    from sas_amd import _lib
    for base in ("plain", "lcp"):  # the reference's binary_search from the table's range
        got = idx.search_batch(dbuf, doff, dlen, algo=base, flags=_lib.SAS_PREFIX_RANGE).cpu().numpy()
        assert np.array_equal(got, res["plain"]), base
    lo, hi = idx.search_range(dbuf, doff, dlen)
    lo = lo.cpu().numpy()
    for k in rng.choice(len(qs), 3000, replace=False):
        q = bytes(qs[k])
        r = int(lo[k])
        cur = int(idx.suffix_array(count=1, start=r)[0]) if r < n else n
        assert int(res["plain"][k]) == cur
        if r < n:
            assert bytes(ht[cur:cur + len(q)]) >= q
        if r > 0:
            prev = int(idx.suffix_array(count=1, start=r - 1)[0])
            assert bytes(ht[prev:prev + len(q)]) < q


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_multi_device_handle(sas, devices):
    """sas_build_multi / sas_search_multi, REPLICATE and SHARD, with the
    one GPU listed several times: positions equal one whole index / the oracle on a
    random and a repeat-rich text, ragged mixed queries incl. misses and text ends."""
    rng = np.random.default_rng(len(devices))
    blk = rng.integers(0, 4, 4000, dtype=np.uint8)
    for t in (sas.random_string(300_017, seed=3), np.concatenate([blk, blk, rng.integers(0, 4, 777, dtype=np.uint8),
                                                                    blk, blk[:1500]])):
        n = len(t)
        whole = sas.SaNaive.build(t, lcp=False, stree=False, sector=False)
        sa = whole.suffix_array()
        qs = [t[o:o + l] for o, l in zip(rng.integers(0, n - 300, 1500), rng.integers(1, 300, 1500))]
        qs += [rng.integers(0, 4, rng.integers(0, 40), dtype=np.uint8) for _ in range(500)]
        qs += [np.full(k, 3, np.uint8) for k in (1, 32, 100)] + [t[n - k:] for k in (1, 7, 40)]
        buf, off, lens = pack(qs)
        expect = oracle_positions(t, sa, buf, off, lens)
        for mode in ("replicate", "shard"):
            M = sas.SaMulti.build(t, devices, mode=mode)
            assert M.parts() == len(devices)
            if mode == "shard":
                st = [M.stats(g) for g in range(len(devices))]
                assert sum(s["sa_entries"] for s in st) == n
                assert [s["rank_lo"] for s in st] == sorted(s["rank_lo"] for s in st)
            for algo in ("quad", "plain", "prefix"):
                got = M.search_batch(buf, off, lens, algo=algo)
                assert np.array_equal(got, expect), (mode, algo, len(devices), n)
            M.free()


def test_occurrence_ranges_inline_slots(sas):
    """k_sa_prefix2_range: on two- and four-suffix inline prefix tables the lane group tests
    both bounds on the entry's slots, then bisects what is left.  Ranges equal the oracle's
    and the plain bisection's (SAS_RANGE_NO_INLINE) for: p from 4 (ranges far larger than an
    entry: the bisections) to 12 (mostly one entry), fixed lengths below p, at 32 and above
    (text compares), ragged mixes, misses, above-every-suffix and empty queries, a repetitive
    text, a 40-bit SA, host and device pointers (sas_search_range_fixed)."""
    import torch
    from sas_amd import _lib
    rng = np.random.default_rng(44)
    texts = [sas.random_string(200_003, seed=9), np.tile(rng.integers(0, 4, 7, dtype=np.uint8), 20_000)]
    for t in texts:
        n = len(t)
        tp = O.padded(t)
        for p, inl, sa40 in ((4, 2, False), (8, 4, False), (12, 2, False), (10, 2, True), (12, 4, False)):
            idx = sas.SaNaive.build(t, lcp=False, stree=False, sector=False, llcp=False, quad=True, prefix=p,
                                    prefix_inline=inl, sa40=sa40)
            sa = np.ascontiguousarray(idx.suffix_array(), np.uint32)
            for m in (3, 8, 32, 40):
                offs = rng.integers(0, n - m, 1500)
                qb = np.concatenate([t[o:o + m] for o in offs] + [rng.integers(0, 4, 500 * m, dtype=np.uint8),
                                                                  np.full(m, 3, np.uint8)])
                nq = len(qb) // m
                lo, hi = idx.search_range_fixed(qb, m)
                lo2, hi2 = idx.search_range_fixed(qb, m, flags=_lib.SAS_RANGE_NO_INLINE)
                assert np.array_equal(lo, lo2) and np.array_equal(hi, hi2), (n, p, inl, m)
                dlo, dhi = idx.search_range_fixed(torch.from_numpy(qb).cuda(), m)
                assert np.array_equal(dlo.cpu().numpy().astype(np.uint64), lo), (n, p, inl, m)
                assert np.array_equal(dhi.cpu().numpy().astype(np.uint64), hi), (n, p, inl, m)
                for k in list(range(0, nq, 37)) + [nq - 1]:
                    q = qb[k * m:(k + 1) * m]
                    assert (int(lo[k]), int(hi[k])) == O.prefix_range(tp, n, sa, q), (n, p, inl, m, k)
            qs = [t[o:o + l] for o, l in zip(rng.integers(0, n - 300, 800), rng.integers(0, 300, 800))]
            qs += [rng.integers(0, 4, l, dtype=np.uint8) for l in rng.integers(0, 40, 300)]
            qs += [np.zeros(0, np.uint8), np.full(200, 3, np.uint8)]
            buf, off, lens = pack(qs)
            lo, hi = idx.search_range(buf, off, lens)
            lo2, hi2 = idx.search_range(buf, off, lens, flags=_lib.SAS_RANGE_NO_INLINE)
            assert np.array_equal(lo, lo2) and np.array_equal(hi, hi2), (n, p, inl)
            for k in range(0, len(qs), 7):
                assert (int(lo[k]), int(hi[k])) == O.prefix_range(tp, n, sa, qs[k]), (n, p, inl, k)


def test_blocked_pivot_levels(sas):
    """The pivot depth (SAS_BUILD_TOP2_LEVELS): prefix-relative blocks of up to 4 levels, the
    first 15 levels staged in LDS, the depth rounded up to the grid past them and clamped to
    the 25 iterations of an n = 3 x 2^23 text.  Every depth (blocks of 1..4 levels, none at
    all) gives PLAIN, LCP, LLCP and INLINE the positions and probe counts of the oracle's
    binary_search (sas/sa_search.rs:98-112), and sas_stats top2_bytes / rel_bytes are the
    layout's sizes."""
    import bench
    n = 3 << 23
    t = sas.random_string(n, seed=123)
    rng = np.random.default_rng(9)
    nq, m = 20_000, 40
    offs = rng.integers(0, n - m, nq)
    qs = np.stack([t[o:o + m] for o in offs])
    qs[: nq // 4] = rng.integers(0, 4, (nq // 4, m))
    qb = qs.reshape(-1).copy()
    ref = None
    for L in (0, 5, 13, 14, 15, 16, 17, 18, 21, 24, 25):
        idx = sas.SaNaive.build(t, lcp=True, stree=False, sector=False, quad=True, llcp=True, prefix=False,
                                top2_levels=L)
        st = idx.stats()
        R = bench.rel_levels(st["iterations"], 27 if L == 0 else L)
        assert st["top_levels"] == min(R, 15) and st["rel_levels"] == R and st["top2_levels"] == R, \
            (L, st["top_levels"], st["rel_levels"])
        assert st["top2_bytes"] == 0 and st["rel_bytes"] == bench.rel_bytes(R), L
        if ref is None:
            sa = idx.suffix_array()
            tp = O.padded(t)
            ref = np.array([O.search_one(tp, n, sa, q)[0] for q in qs[::50]], np.uint64)
            ref_all, ref_pr = idx.search_fixed(qb, m, algo="plain", probes=True)
            assert np.array_equal(ref_all[::50], ref)
        for algo in ("plain", "lcp", "llcp", "inline"):
            got, pr = idx.search_fixed(qb, m, algo=algo, probes=True)
            assert np.array_equal(got, ref_all), (L, algo)
            assert np.array_equal(pr, ref_pr), (L, algo)
        idx.free()
    # the groups: 4 levels each (a 3-level one ends the LDS part at 15), the last one clamped
    assert [(d, h) for d, h, _ in bench.rel_groups(27)] == [(0, 4), (4, 4), (8, 4), (12, 3), (15, 4), (19, 4), (23, 4)]
    assert [(d, h) for d, h, _ in bench.rel_groups(25)][-1] == (23, 2)
    assert [(d, h) for d, h, _ in bench.rel_groups(5)] == [(0, 4), (4, 1)]


def test_rel_pivot_blocks(sas):
    """The prefix-relative pivot blocks (common.hpp SAS_REL_GROUP): a block decides its 4
    levels from the 8 chars after its bounds' common prefix P (capped at 24).  Texts with
    planted repeats of 10..45 chars (P near and past the cap, 8-char ties) and a periodic text
    (every P capped, every key a tie), queries of every length 0..40 plus 64 and 100 (m < P + 8
    included), one-char mutations at every offset, negatives and text-end suffixes: PLAIN,
    LCP, LLCP and INLINE equal the oracle's binary_search (sas/sa_search.rs:98-112) and PLAIN
    without the pivot levels, positions (and probe counts, where they follow it)."""
    import bench
    from sas_amd import _lib
    rng = np.random.default_rng(21)
    base = sas.random_string(3 << 20, seed=99)
    planted = base.copy()
    n0 = len(planted)
    for a, b, ln in zip(rng.integers(0, n0 - 64, 60_000), rng.integers(0, n0 - 64, 60_000),
                        rng.integers(10, 46, 60_000)):
        planted[b:b + ln] = planted[a:a + ln]
    texts = {"planted": planted, "period_9": np.tile(rng.integers(0, 4, 9, dtype=np.uint8), (1 << 17) // 9 + 5)}
    for name, t in texts.items():
        n = len(t)
        idx = sas.SaNaive.build(t, lcp=True, stree=True, sector=False, quad=True, llcp=True, prefix=False)
        st = idx.stats()
        assert st["rel_levels"] == bench.rel_levels(st["iterations"], 27) and st["rel_bytes"] > 0, name
        sa = idx.suffix_array()
        qs = []
        for m in list(range(0, 41)) + [64, 100]:
            for o in rng.integers(0, n - m - 1, 60):
                q = t[o:o + m].copy()
                qs.append(q)
                if m:
                    k = int(rng.integers(0, m))
                    mq = q.copy()
                    mq[k] = (mq[k] + 1 + rng.integers(0, 3)) % 4
                    qs.append(mq)
        qs += [rng.integers(0, 4, l, dtype=np.uint8) for l in rng.integers(0, 40, 300)]
        qs += [t[n - k:] for k in (1, 2, 7, 8, 9, 24, 31, 32, 33)]
        qs += [np.concatenate([t[n - k:], np.zeros(j, np.uint8)]) for k in (3, 20, 30) for j in (1, 5, 12)]
        buf, qo, ql = pack(qs)
        expect = oracle_positions(t, sa, buf[:-64], qo, ql)
        got, pr = idx.search_batch(buf, qo, ql, algo="plain", probes=True)
        bad = np.nonzero(got != expect)[0]
        assert len(bad) == 0, (name, bad[:5], [qs[i] for i in bad[:2]])
        got0, pr0 = idx.search_batch(buf, qo, ql, algo="plain", probes=True, flags=_lib.SAS_NO_LDS_TOP)
        assert np.array_equal(got0, expect), name
        assert np.array_equal(pr, pr0), name
        # LCP / LLCP take exact lcps off the same keys (a key below q that may end in padding
        # reads the whole entry); INLINE decides on them with the sector predicate
        # STREE_LLCP: the S-tree's run of equal 16-char keys, then LLCP over it (long runs here);
        # QUAD_LLCP: the same inside the run of q's 32-char key (or its 16-char run)
        for algo in ("lcp", "llcp", "inline", "stree_llcp", "quad_llcp"):
            ga, pa = idx.search_batch(buf, qo, ql, algo=algo, probes=True)
            bad = np.nonzero(ga != expect)[0]
            assert len(bad) == 0, (name, algo, bad[:5], [qs[i] for i in bad[:2]])
            if algo in ("lcp", "llcp"):
                assert np.array_equal(pa, pr), (name, algo)
        idx.free()


def test_plain_sa_run_at_array_end(sas):
    """PLAIN over a u32 SA loads the 16-B chunks covering its last <= 8 ranks at once; with
    sa_n % 4 != 0 the chunk of rank sa_n - 1 runs past the SA's last word, so the build pads
    the u32 SA (whole and shard copies) to a 16-B multiple (round 5).  Queries
    whose lower bound lies in the last ranks, or past them (sentinel n), on texts of every
    n % 4 and on shards whose rank count is not a multiple of 4: positions equal the oracle's."""
    rng = np.random.default_rng(77)
    for n in (4099, 4101, 4102, 65537, 65538, 65539):
        t = rng.integers(0, 4, n, dtype=np.uint8)
        t[-40:] = 3  # the largest suffixes: a run of 3s at the end
        sa = O.build_sa(t)
        qs = [np.full(k, 3, np.uint8) for k in range(1, 45)]  # near and past the top of the SA
        qs += [np.concatenate([np.full(k, 3, np.uint8), [j]]).astype(np.uint8) for k in (5, 20, 39) for j in range(4)]
        qs += [t[o:o + 32] for o in rng.integers(0, n - 32, 500)]
        buf, off, lens = pack(qs)
        expect = oracle_positions(t, sa, buf[:-64], off, lens)
        whole = sas.SaNaive.build(t, lcp=False, stree=False, sector=False, quad=False, llcp=False, prefix=False)
        assert whole.stats()["sa_width"] == 4
        assert np.array_equal(whole.search_batch(buf, off, lens, algo="plain"), expect), n
        # a shard of the top ranks, its rank count not a multiple of 4
        lo = n - (n // 3) - (n % 4 == 0)
        shard = sas.SaNaive.build(t, sa=sa, rank_range=(lo, n), lcp=False, stree=False, sector=False, quad=False,
                                  llcp=False, prefix=False)
        got = shard.search_batch(buf, off, lens, algo="plain")
        # queries whose global lower bound lies in the shard (rank >= lo, the boundary rank
        # included) get the same answer; those below it get the shard's clamped lower bound,
        # rank 0 of the shard = SA[lo]
        rank_of = {int(p): r for r, p in enumerate(sa)}
        rk = np.array([rank_of.get(int(p), n) for p in expect])
        sel = rk >= lo
        assert np.array_equal(got[sel], expect[sel]), n
        below = rk < lo
        assert below.any(), n
        assert (got[below] == sa[lo]).all(), n


def test_quad_llcp_runs(sas):
    """SAS_ALGO_QUAD_LLCP (k_sa_quad_llcp): QUAD's descent, then LLCP skipping inside the run of
    q's 32-char key where the routed leaf does not settle it.  A text of 64 copies of a random
    block with 1% substitutions per copy (the bench's lcp_long repetitive shape, small): runs of
    equal 32-char keys span many leaves, q's key run and 16-char run differ, and the path of the
    next 16-char key parts from q's at various levels.  Positive queries of 33..300 chars,
    one-char mutations past char 16 and past char 32, text-end suffixes shorter than 32 chars
    inside runs, and a ragged mix with queries of <= 32 chars: positions equal the oracle's
    binary_search (sas/sa_search.rs:98-112) and PLAIN's.  A relative-layout quad tree is
    refused (EINVAL)."""
    from sas_amd import _lib
    rng = np.random.default_rng(5)
    blk = sas.random_string(1 << 14, seed=7)
    copies = []
    for _ in range(64):
        c = blk.copy()
        k = rng.integers(0, len(c), len(c) // 100)
        c[k] = rng.integers(0, 4, len(k), dtype=np.uint8)
        copies.append(c)
    t = np.concatenate(copies)
    n = len(t)
    idx = sas.SaNaive.build(t, lcp=True, stree=False, sector=False, quad=True, llcp=True, prefix=False)
    assert idx.stats()["quad_fan"] == 17
    sa = idx.suffix_array()
    qs = []
    for m in (33, 40, 48, 63, 64, 65, 100, 128, 129, 200, 256, 300):
        for o in rng.integers(0, n - m - 1, 400):
            q = t[o:o + m].copy()
            qs.append(q)
            for k in (int(rng.integers(16, 32)), int(rng.integers(32, m))):
                mq = q.copy()
                mq[k] = (mq[k] + 1 + rng.integers(0, 3)) % 4
                qs.append(mq)
    for k in (1, 5, 17, 31, 32, 33, 40):
        tail = t[n - k:]
        qs += [np.concatenate([tail, np.zeros(j, np.uint8)]) for j in (0, 1, 40) if k + j > 32]
        qs += [np.concatenate([tail, np.full(40, 3, np.uint8)])]
    qs += [t[o:o + m] for o, m in zip(rng.integers(0, n - 40, 2000), rng.integers(0, 33, 2000))]  # <= 32
    order = rng.permutation(len(qs))
    qs = [qs[i] for i in order]
    buf, qo, ql = pack(qs)
    expect = oracle_positions(t, sa, buf[:-64], qo, ql)
    got = idx.search_batch(buf, qo, ql, algo="quad_llcp")
    bad = np.nonzero(got != expect)[0]
    assert len(bad) == 0, (bad[:5], [qs[i][:40] for i in bad[:2]])
    assert np.array_equal(got, idx.search_batch(buf, qo, ql, algo="plain"))
    # fixed-length batches (the lcp_long shape) through the device path
    import torch
    for m in (64, 256):
        off = rng.integers(0, n - m - 1, 5000)
        qb = np.concatenate([t[o:o + m] for o in off])
        exp_m = oracle_positions(t, sa, qb, np.arange(len(off), dtype=np.uint64) * m, np.full(len(off), m, np.uint32))
        dq = torch.from_numpy(qb).cuda()
        assert np.array_equal(idx.search_fixed(dq, m, algo="quad_llcp").cpu().numpy().astype(np.uint64), exp_m), m
    idx.free()
    rel = sas.SaNaive.build(t[: 1 << 16], lcp=True, stree=False, sector=False, llcp=True, prefix=False,
                            flags=_lib.SAS_BUILD_QUAD_REL)
    assert rel.stats()["quad_fan"] == 31
    rb, ro, rl = pack([t[:40]])
    with pytest.raises(sas.SasError):
        rel.search_batch(rb, ro, rl, algo="quad_llcp")
    rel.free()


def test_collect_grid_stride(sas):
    """k_bucket_count / k_bucket_collect stride over their chunks (a dispatch holds < 2^32
    work-items: the n = 2^36 part build of round 5 failed with "invalid configuration"
    before).  SAS_COLLECT_GRID caps the grid so that a 2^22-char text takes the same stride
    loop: the 40-bit whole and part builds through the capped grid equal the uncapped ones."""
    n = (1 << 22) + 12345
    t = sas.random_string(n, seed=4)
    kw = dict(lcp=False, stree=False, sector=False, quad=False, llcp=False, prefix=False)
    ref = sas.SaNaive.build(t, sa40=True, **kw)
    sa_ref = ref.suffix_array()
    ref.free()
    refp = sas.SaNaive.build_part(t, 1, 3, **kw)
    part_ref = refp.suffix_array()
    refp.free()
    old = os.environ.get("SAS_COLLECT_GRID")
    try:
        for g in ("1", "3", "7"):
            os.environ["SAS_COLLECT_GRID"] = g
            idx = sas.SaNaive.build(t, sa40=True, verify=True, **kw)
            assert np.array_equal(idx.suffix_array(), sa_ref), g
            idx.free()
            part = sas.SaNaive.build_part(t, 1, 3, **kw)
            assert np.array_equal(part.suffix_array(), part_ref), g
            part.free()
    finally:
        if old is None:
            os.environ.pop("SAS_COLLECT_GRID", None)
        else:
            os.environ["SAS_COLLECT_GRID"] = old
    assert O.check_sa(t, sa_ref) == 0


def test_llcp_tails_short_suffixes_and_probes(sas):
    """The two LLCP tails (STREE_LLCP: runs of equal 16-char keys; QUAD_LLCP: of equal 32-char
    keys, or 16-char ones) substitute an entry's own Llcp / Rlcp for a run bound no compare
    measured; a text-end suffix shorter than the key inside or beside a run is the case where
    that substitute falls below the true lcp.  A periodic text ending in a short
    aperiodic tail and a run of As (text-end suffixes of 1..40 chars whose zero-padded keys
    equal their neighbours'), queries that are those suffixes (zero-padded and not), queries of
    m < 16, and mutations: positions equal the oracle's binary_search.  out_probes of the tree
    algorithms counts memory reads, not the reference's cnt (include/sas.h): every lookup
    reads at least its descent and leaf, and at most the descent(s), the leaf extension and
    one LLCP entry per binary-search level."""
    rng = np.random.default_rng(12)
    per = rng.integers(0, 4, 23, dtype=np.uint8)
    t = np.concatenate([np.tile(per, 4000), rng.integers(0, 4, 7, dtype=np.uint8), per[:9],
                        np.zeros(20, np.uint8), per[:5], np.zeros(3, np.uint8)])
    n = len(t)
    idx = sas.SaNaive.build(t, lcp=True, stree=True, sector=False, quad=True, llcp=True, prefix=False)
    st = idx.stats()
    sa = idx.suffix_array()
    qs = []
    for k in range(1, 41):
        tail = t[n - k:]
        qs += [tail, np.concatenate([tail, np.zeros(3, np.uint8)]), np.concatenate([tail, [1]]).astype(np.uint8)]
    qs += [t[o:o + m] for o, m in zip(rng.integers(0, n - 70, 1500), rng.integers(1, 16, 1500))]
    qs += [t[o:o + m] for o, m in zip(rng.integers(0, n - 70, 1500), rng.integers(16, 70, 1500))]
    for q in list(qs[-400:]):
        mq = q.copy()
        mq[int(rng.integers(0, len(mq)))] ^= 1
        qs.append(mq)
    buf, qo, ql = pack(qs)
    expect = oracle_positions(t, sa, buf[:-64], qo, ql)
    lvl = int(np.ceil(np.log2(n))) + 2
    for algo, layers in (("stree_llcp", st["stree_layers"]), ("quad_llcp", st["quad_layers"])):
        got, pr = idx.search_batch(buf, qo, ql, algo=algo, probes=True)
        bad = np.nonzero(got != expect)[0]
        assert len(bad) == 0, (algo, bad[:5], [qs[i] for i in bad[:2]])
        assert (pr >= layers).all(), (algo, int(pr.min()))
        assert (pr <= 2 * layers + 4 + lvl + 2).all(), (algo, int(pr.max()))
    idx.free()
