"""GPU parity of SAS_ALGO_INTERP (interpolation_search<16>, sas/sa_search.rs:376-421) and of
the tagged index (SAS_BUILD_TAGGED + SAS_ALGO_TAGGED, the configs[3] path) against the oracle.

Bar: bit-exact positions for every query; INTERP's out_probes equal the restated
interpolation_search's `cnt` (oracle/sa_oracle.c orc_interpolation_search, itself pinned to
binary_search's positions on the definition fixtures); TAGGED's out_probes equal the
reference's binary_search `cnt` with the prefix table live (sas/sa_search.rs:86-112);
occurrence ranges equal the oracle's.
"""
import numpy as np
import pytest

from oracle import pyoracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sas():
    import sas_amd
    return sas_amd


def pack(qs):
    lens = np.array([len(q) for q in qs], np.uint32)
    off = np.zeros(len(qs), np.uint64)
    if len(qs) > 1:
        off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = np.concatenate([np.asarray(q, np.uint8) for q in qs] + [np.zeros(64, np.uint8)])
    return buf, off, lens


def mixed_queries(t, rng, nq=3000):
    n = len(t)
    qs = [t[o:o + l] for o, l in zip(rng.integers(0, max(1, n - 300), nq), rng.integers(0, 300, nq))]
    qs += [rng.integers(0, 4, rng.integers(0, 60), dtype=np.uint8) for _ in range(nq // 4)]  # misses
    qs += [np.concatenate([t[o:o + 20], [3, 3]]).astype(np.uint8) for o in rng.integers(0, max(1, n - 30), 100)]
    qs += [np.concatenate([t[n - k:], np.zeros(j, np.uint8)]) for k in (1, 3, 13, 28, 29, 40) if k <= n
           for j in (0, 2)]  # text-end suffixes, with zeros (the A7 edge case)
    qs += [np.zeros(0, np.uint8), np.full(40, 3, np.uint8), np.zeros(n + 5, np.uint8)[:300]]
    return qs


def texts(rng):
    blk = rng.integers(0, 4, 3000, dtype=np.uint8)
    return {
        "random": O.random_string(200_003, seed=5),
        "all_A": np.zeros(30_000, np.uint8),
        "period_5": np.tile(rng.integers(0, 4, 5, dtype=np.uint8), 9000),
        "repeats": np.concatenate([blk, rng.integers(0, 4, 77, dtype=np.uint8), blk, blk[:2000], blk]),
        "A_run_end": np.concatenate([rng.integers(0, 4, 20_000, dtype=np.uint8), np.zeros(500, np.uint8)]),
    }


def expected(t, sa, qs):
    """(positions, lower-bound ranks) from the oracle's binary_search."""
    tp = O.padded(t)
    pos = np.array([O.search_one(tp, len(t), sa, q)[0] for q in qs], np.uint64)
    rank = np.array([O.lower_bound_rank(tp, len(t), sa, q) for q in qs], np.uint64)
    return pos, rank


def table_cnt(t, sa, qs, rank, p):
    """The reference's cnt with the prefix table live (sas/sa_search.rs:86-112): 1 for the
    table, then binary_search's iterations over [table[K], table[K+1]) ending at the
    lower bound rank."""
    n = len(t)
    tp = O.padded(t).astype(np.int64)
    keys = np.zeros(n, np.int64)
    for j in range(p):
        keys = keys * 4 + tp[sa.astype(np.int64) + j]
    out = []
    for q, r in zip(qs, rank):
        qq = np.zeros(p, np.int64)
        qq[: min(p, len(q))] = np.asarray(q[:p], np.int64)
        K = int(np.polyval(qq, 4)) if p else 0
        lo = int(np.searchsorted(keys, K, "left"))
        hi = int(np.searchsorted(keys, K + 1, "left"))
        c = 1
        while lo < hi:
            mid = (lo + hi) // 2
            if mid < r:
                lo = mid + 1
            else:
                hi = mid
            c += 1
        out.append(c)
    return np.array(out, np.uint32)


# ------------------------------------------------------------------ INTERP
def test_interp_positions_and_cnt(sas):
    """Fused-leaf probes (quad built) and SA + text probes (u32 and 40-bit SA) give the
    oracle's positions and its interpolation_search cnt, query by query."""
    rng = np.random.default_rng(12)
    for name, t in texts(rng).items():
        n = len(t)
        sa = O.build_sa(t)
        qs = mixed_queries(t, rng, 1500)
        qs = [q for q in qs if len(q) >= 16] + [q for q in qs if len(q) < 16][:200]
        buf, off, lens = pack(qs)
        tp = O.padded(t)
        exp = [O.interpolation_search(tp, n, sa, q) for q in qs]
        epos = np.array([e[0] for e in exp], np.uint64)
        ecnt = np.array([e[1] for e in exp], np.uint32)
        assert np.array_equal(epos, expected(t, sa, qs)[0]), name  # same result as binary_search
        for kw in ({}, {"quad": False}, {"quad": False, "sa40": True}):
            idx = sas.SaNaive.build(t, lcp=False, stree=False, sector=False, llcp=False, **kw)
            got, cnt = idx.search_batch(buf, off, lens, algo="interp", probes=True)
            bad = np.nonzero(got != epos)[0]
            assert len(bad) == 0, (name, kw, bad[:5])
            bad = np.nonzero(cnt != ecnt)[0]
            assert len(bad) == 0, (name, kw, bad[:5], cnt[bad[:5]], ecnt[bad[:5]])


def test_interp_c0_shape_and_range_flag(sas):
    """configs[0] (1 MiB ChaCha8 text, 10^4 x len-16): the reference's own interpolation
    run (main.rs:97).  With SAS_PREFIX_RANGE it starts from the prefix table's range."""
    from sas_amd import _lib
    n, nq, m = 1 << 20, 10_000, 16
    t = sas.random_string(n)
    sa = O.build_sa(t)
    off, _, _ = sas.random_queries(n, nq, len_lo=m, len_hi=m + 1)
    qb = np.concatenate([t[o:o + m] for o in off.astype(np.int64)])
    tp = O.padded(t)
    exp = [O.interpolation_search(tp, n, sa, qb[k * m:(k + 1) * m]) for k in range(nq)]
    idx = sas.SaNaive.build(t, lcp=False, stree=False, sector=False, llcp=False, prefix=8)
    got, cnt = idx.search_fixed(qb, m, algo="interp", probes=True)
    assert np.array_equal(got, np.array([e[0] for e in exp], np.uint64))
    assert np.array_equal(cnt, np.array([e[1] for e in exp], np.uint32))
    assert 4 < cnt.mean() < 12  # ~8 probes per lookup vs binary search's 21
    got2, cnt2 = idx.search_fixed(qb, m, algo="interp", probes=True, flags=_lib.SAS_PREFIX_RANGE)
    assert np.array_equal(got2, got) and (cnt2 >= 1).all()


def test_tagged_index_serves_its_algos(sas):
    from sas_amd._lib import SasError
    idx = sas.SaNaive.build(O.random_string(5000), tagged=True)
    got = idx.search([np.array([1, 2, 3], np.uint8)], algo="interp")  # n < 2^32: served
    assert got.shape == (1,)
    with pytest.raises(SasError):
        idx.search([np.array([1], np.uint8)], algo="quad")  # no tree on a tagged index


# ------------------------------------------------------------------ TAGGED
@pytest.mark.parametrize("p", [None, 1, 3, 9])
def test_tagged_matches_oracle(sas, p):
    """Tagged entries + bucket table for several p (1: huge buckets, the bisection past
    the window; 9: tiny ones), u32- and 40-bit-built SAs, on random and repeat-rich texts:
    positions, cnt, ranges, the SA itself; PLAIN / LCP / INTERP on the same index."""
    rng = np.random.default_rng(40 + (p or 0))
    for name, t in texts(rng).items():
        n = len(t)
        sa = O.build_sa(t)
        qs = mixed_queries(t, rng)
        buf, off, lens = pack(qs)
        epos, erank = expected(t, sa, qs)
        for sa40 in (False, True):
            idx = sas.SaNaive.build(t, tagged=True if p is None else p, sa40=sa40, verify=True, lcp=False)
            st = idx.stats()
            assert st["sa_width"] == 8 and st["tag_chars"] >= 1
            assert st["tag_table_bytes"] == (4 ** st["tag_chars"] + 1) * 8
            assert np.array_equal(idx.suffix_array(), sa.astype(np.uint64)), name
            idx.verify()
            got, cnt = idx.search_batch(buf, off, lens, algo="tagged", probes=True)
            bad = np.nonzero(got != epos)[0]
            assert len(bad) == 0, (name, p, sa40, bad[:5], [qs[i] for i in bad[:2]])
            ecnt = table_cnt(t, sa, qs, erank, st["tag_chars"])
            assert np.array_equal(cnt, ecnt), (name, p, np.nonzero(cnt != ecnt)[0][:5])
            for algo in ("plain", "lcp", "interp"):
                assert np.array_equal(idx.search_batch(buf, off, lens, algo=algo), epos), (name, algo)
            lo, hi = idx.search_range(buf, off, lens)
            tp = O.padded(t)
            for k in range(0, len(qs), 7):
                assert (int(lo[k]), int(hi[k])) == O.prefix_range(tp, n, sa, qs[k]), (name, k)


@pytest.mark.parametrize("p", [None, 1, 3, 7])
def test_tag_lines_match_oracle(sas, p):
    """Bucket lines (SAS_BUILD_TAG_LINES) for several p (1: a few huge buckets, every lookup
    in the overflow array; 7: ~1-12 suffixes a line, slots past the count), u32- and
    40-bit-built SAs, on random and repeat-rich texts: positions, cnt, ranges and the SA
    equal the oracle's and the rank-ordered tagged index's; no SA array behind it."""
    rng = np.random.default_rng(60 + (p or 0))
    for name, t in texts(rng).items():
        n = len(t)
        sa = O.build_sa(t)
        qs = mixed_queries(t, rng)
        buf, off, lens = pack(qs)
        epos, erank = expected(t, sa, qs)
        for sa40 in (False, True):
            idx = sas.SaNaive.build(t, tagged=True if p is None else p, sa40=sa40, verify=True, lcp=False,
                                    tag_lines=True)
            st = idx.stats()
            pp = st["tag_chars"]
            assert st["tag_line_slots"] == 20 and st["tag_table_bytes"] == 4 ** pp * 128 + (4 ** pp + 1) * 8
            assert st["tag_line_tag_bits"] == 48 - max(32, n.bit_length())  # 16 below 2^32
            assert st["sa_bytes"] == st["tag_overflow_entries"] * 8 and st["text2_bytes"] == st["text_bytes"]
            assert np.array_equal(idx.suffix_array(), sa.astype(np.uint64)), name
            got, cnt = idx.search_batch(buf, off, lens, algo="tagged", probes=True)
            bad = np.nonzero(got != epos)[0]
            assert len(bad) == 0, (name, p, sa40, bad[:5], [qs[i] for i in bad[:2]])
            ecnt = table_cnt(t, sa, qs, erank, pp)
            assert np.array_equal(cnt, ecnt), (name, p, np.nonzero(cnt != ecnt)[0][:5])
            lo, hi = idx.search_range(buf, off, lens)
            tp = O.padded(t)
            for k in range(0, len(qs), 7):
                assert (int(lo[k]), int(hi[k])) == O.prefix_range(tp, n, sa, qs[k]), (name, k)
            for algo in ("plain", "lcp", "interp"):
                with pytest.raises(sas.SasError):
                    idx.search_batch(buf, off, lens, algo=algo)
            with pytest.raises(sas.SasError):
                idx.verify()
            # overflow entries: ranks first + 20 .. first + count of each bucket of >= 20
            keys = np.zeros(n, np.int64)
            tpi = tp.astype(np.int64)
            for j in range(pp):
                keys = keys * 4 + tpi[sa.astype(np.int64) + j]
            c = np.bincount(keys, minlength=4 ** pp)
            assert st["tag_overflow_entries"] == int(np.sum(np.where(c >= 20, c - 19, 0))), name
            idx.free()


def test_tagged_device_ragged_and_validation(sas):
    """Device-pointer ragged batches (odd offsets, no slack after the last query) and
    SAS_VALIDATE: a bad code anywhere in a query -- including past the words the kernel
    keeps in registers (char 200 of a 250-char query) -- fails with EINVAL."""
    import torch
    from sas_amd import _lib
    from sas_amd._lib import SasError
    t = O.random_string(300_007, seed=8)
    idx = sas.SaNaive.build(torch.from_numpy(t).cuda(), tagged=True)
    rng = np.random.default_rng(4)
    lens = rng.integers(0, 300, 5000).astype(np.uint32)
    starts = rng.integers(0, len(t) - 300, 5000)
    qs = [t[s:s + l] for s, l in zip(starts, lens)]
    buf = np.concatenate([np.array([1, 2, 3], np.uint8)] + qs)
    off = (np.concatenate([[0], np.cumsum(lens[:-1])]) + 3).astype(np.uint64)
    expect = expected(t, O.build_sa(t), qs)[0]
    got = idx.search_batch(torch.from_numpy(buf).cuda(), torch.from_numpy(off.view(np.int64)).cuda(),
                           torch.from_numpy(lens.view(np.int32)).cuda(), algo="tagged")
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().astype(np.uint64), expect)
    full = sas.SaNaive.build(t)
    for index, algo in ((idx, "tagged"), (full, "prefix"), (full, "quad"), (full, "plain")):
        q = t[1000:1250].copy()
        q[200] = 7
        dq = torch.from_numpy(np.concatenate([q, np.zeros(16, np.uint8)])).cuda()
        doff = torch.zeros(1, dtype=torch.int64, device="cuda")
        dlen = torch.full((1,), 250, dtype=torch.int32, device="cuda")
        with pytest.raises(SasError):
            index.search_batch(dq, doff, dlen, algo=algo, flags=_lib.SAS_VALIDATE)
        with pytest.raises(SasError):  # host pointers always validate
            index.search_batch(np.concatenate([q, np.zeros(16, np.uint8)]), np.zeros(1, np.uint64),
                               np.array([250], np.uint32), algo=algo)
    with pytest.raises(SasError):
        full.search_range(torch.from_numpy(np.concatenate([q, np.zeros(16, np.uint8)])).cuda(),
                          torch.zeros(1, dtype=torch.int64, device="cuda"),
                          torch.full((1,), 250, dtype=torch.int32, device="cuda"), flags=_lib.SAS_VALIDATE)


@pytest.mark.parametrize("lines", [False, True])
def test_tagged_saturated_bucket(sas, lines):
    """A bucket with >= 2^24 suffixes saturates the 24-bit count: the lookup reads the next
    bucket word (the next line's first rank) for its end.  All-A text: SA[r] = n - 1 - r,
    every suffix in bucket 0."""
    import torch
    n = (1 << 24) + 1000
    t = torch.zeros(n, dtype=torch.uint8, device="cuda")
    idx = sas.SaNaive.build(t, tagged=True, lcp=False, tag_lines=lines)
    st = idx.stats()
    p = st["tag_chars"]
    # ceil(log4 n) (minus 2 for lines): 4^12 = 2^24 < n; one bucket holds all n > 2^24 - 1 suffixes
    assert p == (11 if lines else 13)
    sa = idx.suffix_array(count=5)
    assert sa.tolist() == [n - 1 - r for r in range(5)]
    ms = [1, 5, 11, 12, 13, 27, 28, 29, 100, 257, 4000, n, n + 1]
    qs = [np.zeros(m, np.uint8) for m in ms if m < 10_000]
    qs += [np.concatenate([np.zeros(k, np.uint8), [1]]).astype(np.uint8) for k in (0, 3, 30, 500)]
    buf, off, lens = pack(qs)
    got, cnt = idx.search_batch(buf, off, lens, algo="tagged", probes=True)
    for k, q in enumerate(qs):
        m = len(q)
        expect = n - m if not q.any() else n  # 0^m: the shortest suffix of length >= m
        assert int(got[k]) == expect, (k, m)
    lo, hi = idx.search_range(buf, off, lens)
    for k, q in enumerate(qs):
        if not q.any():
            assert (int(lo[k]), int(hi[k])) == (len(q) - 1, n), k


@pytest.mark.parametrize("lines", [False, True])
def test_tagged_wave_staging_paths(sas, lines):
    """k_sa_tagged's wave-staged queries: a contiguous batch (staged through LDS), the same
    queries with shuffled offsets (spans past 16,608 chars fall back to per-lane loads), a wave
    of empty queries, a tail wave of 37 queries, and queries that sit at the very end of the
    device buffer (no slack): every form equals the oracle."""
    import torch
    t = O.random_string(400_009, seed=12)
    n = len(t)
    sa = O.build_sa(t)
    idx = sas.SaNaive.build(torch.from_numpy(t).cuda(), tagged=True, lcp=False, tag_lines=lines)
    rng = np.random.default_rng(3)
    nq = 64 * 40 + 37
    lens = rng.integers(0, 260, nq).astype(np.uint32)
    lens[64:128] = 0  # one wave of empty queries
    starts = rng.integers(0, n - 260, nq)
    qs = [t[s:s + l] for s, l in zip(starts, lens)]
    expect = expected(t, sa, qs)[0]
    buf = np.concatenate(qs).astype(np.uint8)  # no slack after the last query
    off = np.zeros(nq, np.uint64)
    off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    dbuf = torch.from_numpy(buf).cuda()
    for name, o in (("contiguous", off), ("shuffled", None)):
        if o is None:  # the same bytes, queries in a different order: offsets jump around
            perm = rng.permutation(nq)
            o = off[perm]
            ln, ex = lens[perm], expect[perm]
        else:
            ln, ex = lens, expect
        got = idx.search_batch(dbuf, torch.from_numpy(o.view(np.int64)).cuda(),
                               torch.from_numpy(ln.view(np.int32)).cuda(), algo="tagged")
        torch.cuda.synchronize()
        bad = np.nonzero(got.cpu().numpy().astype(np.uint64) != ex)[0]
        assert len(bad) == 0, (name, bad[:5])
    # fixed-length batch whose count is not a multiple of 64 (a tail wave)
    m = 40
    qb = np.concatenate([t[s:s + m] for s in starts[:101]])
    got = idx.search_fixed(torch.from_numpy(qb).cuda(), m, algo="tagged")
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().astype(np.uint64),
                          expected(t, sa, [t[s:s + m] for s in starts[:101]])[0])
    # the largest staged span: 64 queries of 256 chars starting 15 bytes past a 16-B block
    # (16,399 chars, inside the 16,608-char stage), and 64 of 260 chars (past it: per-lane
    # loads); each batch offset into a larger device buffer, with a few misses
    for m, skew in ((256, 15), (256, 1), (260, 15)):
        nq2 = 64 * 3 + 5
        qs2 = [t[s:s + m] for s in starts[:nq2]]
        qs2[7] = rng.integers(0, 4, m, dtype=np.uint8)
        qs2[100] = np.full(m, 3, np.uint8)
        raw = torch.zeros(16 + nq2 * m, dtype=torch.uint8, device="cuda")
        raw[skew:skew + nq2 * m] = torch.from_numpy(np.concatenate(qs2)).cuda()
        o2 = torch.arange(nq2, dtype=torch.int64, device="cuda") * m + skew
        l2 = torch.full((nq2,), m, dtype=torch.int32, device="cuda")
        got = idx.search_batch(raw, o2, l2, algo="tagged")
        torch.cuda.synchronize()
        ex2 = expected(t, sa, qs2)[0]
        bad = np.nonzero(got.cpu().numpy().astype(np.uint64) != ex2)[0]
        assert len(bad) == 0, (m, skew, bad[:5])


@pytest.mark.parametrize("lines", [False, True])
def test_tagged_text_slices(sas, lines):
    """SAS_QUERIES_ARE_SLICES: queries given as slices t[off : off + len] of the indexed text
    (no query bytes; the tie with the query's own suffix skips the text compare) give the
    oracle's positions and the byte queries' probes, on random and repeat-rich texts,
    lengths 0..300 including slices that end at the text's end; a slice past the end is
    EINVAL."""
    import torch
    rng = np.random.default_rng(17)
    for name, t in texts(rng).items():
        n = len(t)
        idx = sas.SaNaive.build(t, lcp=False, tagged=True, tag_lines=lines)
        lens = rng.integers(0, 300, 4000)
        offs = np.array([rng.integers(0, max(1, n - l + 1)) for l in lens], np.int64)
        lens = np.minimum(lens, n - offs)
        offs = np.concatenate([offs, [n - 1, n - 5, n, 0]])
        lens = np.concatenate([lens, [1, 5, 0, min(n, 257)]])
        qs = [t[o:o + l] for o, l in zip(offs, lens)]
        exp, _ = expected(t, np.ascontiguousarray(O.build_sa(t), np.uint32), qs)
        dq_off = torch.from_numpy(offs).cuda()
        dq_len = torch.from_numpy(lens.astype(np.int32)).cuda()
        got, pr = idx.search_slices(dq_off, dq_len, probes=True)
        buf, off, ln = pack(qs)
        byt, bpr = idx.search_batch(buf, off, ln, algo="tagged", probes=True)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy().astype(np.uint64), exp), name
        assert np.array_equal(byt, exp), name
        assert np.array_equal(pr.cpu().numpy().astype(np.uint32), bpr), name
        with pytest.raises(sas.SasError):
            idx.search_slices(torch.tensor([n - 3], dtype=torch.int64, device="cuda"),
                              torch.tensor([4], dtype=torch.int32, device="cuda"))


def test_tag_lines_overflow_heavy(sas):
    """Bucket lines whose answers mostly lie in the overflow array: at p = 2 (~12,500
    suffixes a bucket) every lookup's answer lies past its line's 20 slots (overflow window,
    then the bisection); at p = 5 (~200) both kinds meet in every wave.  60,000 ragged
    queries, byte queries and text slices equal the rank-ordered tagged index's positions,
    and a sample equals the oracle's."""
    import torch
    t = O.random_string(200_003, seed=12)
    n = len(t)
    rng = np.random.default_rng(13)
    nq = 60_000
    off = rng.integers(0, n - 300, nq)
    lens = rng.integers(1, 300, nq).astype(np.uint32)
    qs = [t[o:o + l] for o, l in zip(off, lens)]
    buf, qoff, qlen = pack(qs)
    ref_idx = sas.SaNaive.build(t, tagged=True, lcp=False)
    ref = ref_idx.search_batch(buf, qoff, qlen, algo="tagged")
    ref_idx.free()
    for p in (2, 5):
        idx = sas.SaNaive.build(t, tagged=p, lcp=False, tag_lines=True)
        got = idx.search_batch(buf, qoff, qlen, algo="tagged")
        assert np.array_equal(got, ref), (p, np.nonzero(got != ref)[0][:5])
        src = torch.from_numpy(off.astype(np.int64)).cuda()
        sl = idx.search_slices(src, torch.from_numpy(qlen.astype(np.int32)).cuda())
        torch.cuda.synchronize()
        assert np.array_equal(sl.cpu().numpy().astype(np.uint64), ref.astype(np.uint64)), p
        idx.free()
    sa = O.build_sa(t)
    tp = O.padded(t)
    for k in range(0, nq, 97):
        assert int(ref[k]) == O.search_one(tp, n, sa, qs[k])[0], k


def test_tag_lines_build_holds_only_what_tagged_reads(sas):
    """A bucket-line index serves SAS_ALGO_TAGGED only: the build asks for no LCP array and
    builds no binary-search pivot array (Python turns lcp off; the C ABI refuses LCP / LLCP
    with ENOTSUP and TAG_LINES without TAGGED with EINVAL)."""
    import ctypes as C
    from sas_amd import _lib
    t = sas.random_string(100_003, seed=5)
    idx = sas.SaNaive.build(t, tagged=6, tag_lines=True)  # lcp defaults to True: ignored
    st = idx.stats()
    assert st["lcp_bytes"] == 0 and st["llcp_bytes"] == 0 and st["top2_levels"] == 0
    idx.free()
    h = C.c_void_p()
    base = _lib.SAS_BUILD_TAGGED | _lib.SAS_BUILD_TAG_LINES | _lib.SAS_BUILD_PREFIX_P(6)
    import errno
    for fl, err in ((base | _lib.SAS_BUILD_LCP, errno.ENOTSUP), (_lib.SAS_BUILD_TAG_LINES, errno.EINVAL)):
        rc = _lib.lib().sas_build(t.ctypes.data, len(t), None, 4, fl, C.byref(h))
        assert rc == err, (fl, rc)
