"""Sharded-text mode on the GPU: ShardedSearch over sas_build_part indexes,
fixed-capacity buckets from sas_route_pack_cap, against the whole index.

* ws = 1 through a real RCCL ("nccl") process group, initialised in this process;
* W = 3 parts on one GPU through a loopback exchange (three threads, one per rank, a
  torch.distributed-shaped object that moves the all-to-all chunks between them), so that
  the routing, the bucket layout and the slot gather of a multi-part step run on the GPU.
Bar: positions bit-identical to the whole index's PLAIN search; an overflowing bucket is
redone exactly (check=True) or reported (check=False -> assert_no_overflow raises).
"""
import socket
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sas():
    import sas_amd
    return sas_amd


def queries(t, nq, m, seed):
    rng = np.random.default_rng(seed)
    n = len(t)
    offs = rng.integers(0, n - m, nq)
    qs = np.stack([t[o:o + m] for o in offs])
    qs[: nq // 5] = rng.integers(0, 4, (nq // 5, m))  # negatives
    qs[-1] = 3
    qs[-2] = 0
    return qs.reshape(-1).copy()


def test_sharded_nccl_world1(sas):
    """RCCL process group of one rank: the whole step (route_pack_cap, two equal-split
    all_to_all_single, search, slot gather) with no host synchronisation inside."""
    import torch
    import torch.distributed as dist
    from sas_amd.shard import ShardedSearch
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        n, nq, m = 1_000_003, 50_000, 32
        t = sas.random_string(n, seed=21)
        full = sas.SaNaive.build(t)
        # the part index holds a 40-bit SA; n < 2^32 lets it carry the two-suffix inline table
        part = sas.SaNaive.build_part(torch.from_numpy(t).cuda(), 0, 1, prefix=12, prefix_inline=2)
        qb = queries(t, nq, m, 1)
        expect = full.search_fixed(qb, m, algo="plain")
        dq = torch.from_numpy(qb).cuda()
        for algo, chunks, xself, routed in (("plain", 1, True, False), ("quad", 1, True, False),
                                            ("prefix", 1, True, False), ("prefix", 3, True, False),
                                            ("plain", 2, True, False), ("prefix", 1, False, True),
                                            ("prefix", 2, False, True), ("prefix", 1, False, False),
                                            ("plain", 2, False, False)):
            # prefix: 8-B packed words cross the exchange; chunks > 1: async RCCL pieces;
            # exchange_self: the world-1 exchanges still go through RCCL; routed: route + identity
            # exchange + gather; neither: the world-1 identity step (the lookup alone)
            eng = ShardedSearch(part, dist, 1, 0, torch.device("cuda"), algo=algo, chunks=chunks,
                                exchange_self=xself, routed=routed, max_nq=nq if chunks == 1 else None)
            assert eng.identity == (not xself and not routed)
            assert eng.packed(m) == (algo == "prefix")
            got = eng.search_fixed(dq, m)
            got2 = eng.search_fixed(dq, m, check=False)
            eng.assert_no_overflow()
            exact = eng.search_fixed_exact(dq, m)
            torch.cuda.synchronize()
            for g in (got, got2, exact):
                assert np.array_equal(g.cpu().numpy().astype(np.uint64), expect), algo
        # algorithms sas_search_buckets does not take (the constructor's default STREE,
        # SECTOR, QUAD past 32 chars) search every slot instead of failing with ENOTSUP
        for algo, mm in (("stree", 32), ("sector", 32), ("quad", 64), ("stree", 64)):
            qb2 = qb if mm == m else queries(t, nq, mm, 2)
            exp2 = expect if mm == m else full.search_fixed(qb2, mm, algo="plain")
            eng = ShardedSearch(part, dist, 1, 0, torch.device("cuda"), algo=algo, exchange_self=True, max_nq=nq)
            assert not eng.bucket_lookup(mm), (algo, mm)
            got = eng.search_fixed(torch.from_numpy(qb2).cuda(), mm)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy().astype(np.uint64), exp2), (algo, mm)
        eng = ShardedSearch(part, dist, 1, 0, torch.device("cuda"), exchange_self=True, max_nq=nq)
        assert eng.algo == "stree"
        # a batch larger than the declared max_nq is not refused (a local raise would hang
        # the other ranks in the exchange): with the agreed capacity it is still exact
        eng = ShardedSearch(part, dist, 1, 0, torch.device("cuda"), algo="plain", exchange_self=True,
                            max_nq=nq // 4)
        got = eng.search_fixed(dq, m)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy().astype(np.uint64), expect)
    finally:
        dist.destroy_process_group()


def test_search_buckets_skips_unfilled_slots(sas):
    """sas_search_buckets: bucket b's first counts[b] slots are searched (positions equal
    sas_search_fixed's), the rest are neither read nor written; counts > cap means the
    whole bucket.  Bytes and packed words, PLAIN / QUAD / PREFIX."""
    import torch
    n, m, cap = 300_007, 32, 1000
    t = sas.random_string(n, seed=31)
    idx = sas.SaNaive.build(torch.from_numpy(t).cuda(), prefix=10, prefix_inline=2)
    counts = torch.tensor([0, 1, 999, 1000, 5000, 17], dtype=torch.int64, device="cuda")
    nb = counts.numel()
    qb = torch.from_numpy(queries(t, nb * cap, m, 4)).cuda()
    words = sas.SaNaive.pack_queries(qb, m)
    live = (torch.arange(nb * cap, device="cuda") % cap) < torch.repeat_interleave(counts.clamp(max=cap), cap)
    for algo in ("plain", "quad", "prefix"):
        expect = idx.search_fixed(qb, m, algo=algo)
        for q in ((qb, words) if algo == "prefix" else (qb,)):
            out = torch.full((nb * cap,), -7, dtype=torch.int64, device="cuda")
            idx.search_buckets(q, m, cap, counts, algo=algo, out=out)
            torch.cuda.synchronize()
            assert torch.equal(out[live], expect[live]), algo
            assert bool((out[~live] == -7).all()), algo
            assert int(live.sum()) == 0 + 1 + 999 + 1000 + 1000 + 17
    with pytest.raises(sas.SasError):  # SECTOR has no bounded kernel: ENOTSUP
        idx.search_buckets(qb, m, cap, counts, algo="sector")


def test_c4_record_shape_world1(sas):
    """The configs[4] record's exact shape at N = 1: a 2^30-char text, its one part built
    with sas_build_part and the two-suffix inline table (p = 16), 10^7 len-32 queries
    through ShardedSearch with the packed exchange (RCCL world-1 group, both the forced
    exchange and the default identity), positions bit-identical to the replicated index's
    PREFIX output (built first, searched, freed: the two indexes do not fit together)."""
    import torch
    import torch.distributed as dist
    from sas_amd.shard import ShardedSearch
    n, nq, m = 1 << 30, 10_000_000, 32
    text = sas.random_string(n, seed=31416, device="cuda")
    full = sas.SaNaive.build(text, lcp=False, stree=False, sector=False, llcp=False, prefix=16, prefix_inline=2)
    off = torch.from_numpy(sas.random_queries(n, nq, seed=31416, word_pos=n, margin=200, len_lo=m,
                                              len_hi=m + 1)[0].astype(np.int64)).cuda()
    ar = torch.arange(m, device="cuda", dtype=torch.int64)
    qb = torch.empty(nq * m, dtype=torch.uint8, device="cuda")
    for s0 in range(0, nq, 1 << 18):
        e0 = min(nq, s0 + (1 << 18))
        qb[s0 * m:e0 * m] = text[(off[s0:e0, None] + ar[None, :]).reshape(-1)]
    expect = full.search_fixed(qb, m, algo="prefix")
    torch.cuda.synchronize()
    full.free()
    torch.cuda.empty_cache()
    part = sas.SaNaive.build_part(text, 0, 1, lcp=False, stree=False, sector=False, quad=True, llcp=False,
                                  prefix=16, prefix_inline=2)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        for xself, routed in ((True, False), (False, True), (False, False)):
            eng = ShardedSearch(part, dist, 1, 0, torch.device("cuda"), algo="prefix", max_nq=nq,
                                exchange_self=xself, routed=routed)
            assert eng.packed(m)
            out = torch.empty(nq, dtype=torch.int64, device="cuda")
            for _ in range(2):
                eng.search_fixed(qb, m, check=False, out=out)
            eng.assert_no_overflow()
            torch.cuda.synchronize()
            assert torch.equal(out, expect), (xself, routed)
    finally:
        dist.destroy_process_group()
        part.free()


class Loopback:
    """torch.distributed-shaped exchange between W threads of one process (one per rank);
    every collective is three barriers: deposit, read, done."""

    class ReduceOp:
        MAX = "max"

    def __init__(self, W):
        self.W = W
        self.bar = threading.Barrier(W)
        self.slots = [None] * W

    def _swap(self, rank, item):
        self.slots[rank] = item
        self.bar.wait()
        items = list(self.slots)
        self.bar.wait()
        return items

    def rank(self, r):
        lb = self

        class R:
            ReduceOp = Loopback.ReduceOp

            @staticmethod
            def all_gather(outs, t, group=None):
                items = lb._swap(r, t)
                for i in range(lb.W):
                    outs[i].copy_(items[i])
                lb.bar.wait()

            @staticmethod
            def all_reduce(t, op=None, group=None):
                import torch
                items = lb._swap(r, t.clone())
                t.copy_(torch.stack(items).max(0).values)
                lb.bar.wait()

            @staticmethod
            def all_to_all_single(out, inp, out_splits=None, in_splits=None, group=None, async_op=False):
                items = lb._swap(r, (inp, in_splits))
                pos = 0
                for src in range(lb.W):
                    sin, ssp = items[src]
                    if ssp is None:
                        sz = sin.numel() // lb.W
                        start = r * sz
                    else:
                        start, sz = sum(ssp[:r]), ssp[r]
                    out[pos:pos + sz].copy_(sin[start:start + sz])
                    pos += sz
                lb.bar.wait()  # no rank reuses its send buffer before every copy is queued
                if async_op:  # done already (copies on this rank's stream): a no-op handle

                    class Done:
                        @staticmethod
                        def wait():
                            return True
                    return Done()
        return R


@pytest.mark.parametrize("W", [3])
def test_sharded_parts_loopback(sas, W):
    """W sas_build_part indexes on one GPU, each driven by its own rank thread: routed,
    bucketed, exchanged and gathered answers equal the whole index for every rank's
    queries; a skewed batch into tiny buckets overflows, is redone exactly with
    check=True and reported with check=False."""
    import torch
    from sas_amd.shard import ShardedSearch
    n, nq, m = 2_000_003, 30_000, 24
    t = sas.random_string(n, seed=23)
    full = sas.SaNaive.build(t)
    dt = torch.from_numpy(t).cuda()
    parts = [sas.SaNaive.build_part(dt, g, W, prefix=12, prefix_inline=2) for g in range(W)]
    lb = Loopback(W)
    qbs = [queries(t, nq, m, 10 + r) for r in range(W)]
    expect = [full.search_fixed(q, m, algo="plain") for q in qbs]
    res, errs = {}, []

    def rank_main(r):
        try:
            d = lb.rank(r)
            eng = ShardedSearch(parts[r], d, W, r, torch.device("cuda"), algo="plain")
            dq = torch.from_numpy(qbs[r]).cuda()
            a = eng.search_fixed(dq, m)
            b = eng.search_fixed(dq, m, check=False)
            eng.assert_no_overflow()
            c = eng.search_fixed_exact(dq, m)
            pre = ShardedSearch(parts[r], d, W, r, torch.device("cuda"), algo="prefix")  # packed exchange
            e = pre.search_fixed(dq, m)
            pipe = ShardedSearch(parts[r], d, W, r, torch.device("cuda"), algo="prefix", chunks=3)  # pieces
            e3 = pipe.search_fixed(dq, m)
            tight = ShardedSearch(parts[r], d, W, r, torch.device("cuda"), algo="quad", slack=0.5, min_cap=0)
            skew = torch.from_numpy(np.tile(qbs[r][:m], nq // 10).copy()).cuda()
            sk = tight.search_fixed(skew, m)
            tight.search_fixed(skew, m, check=False)
            raised = False
            try:
                tight.assert_no_overflow()
            except RuntimeError:
                raised = True
            torch.cuda.synchronize()
            res[r] = (a.cpu().numpy(), b.cpu().numpy(), c.cpu().numpy(), sk.cpu().numpy(), raised, e.cpu().numpy(),
                      e3.cpu().numpy())
        except Exception as e:  # surfaced below
            errs.append((r, repr(e)))
            lb.bar.abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(W)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not errs, errs
    for r in range(W):
        a, b, c, sk, raised, e, e3 = res[r]
        for g in (a, b, c, e, e3):
            assert np.array_equal(g.astype(np.uint64), expect[r]), r
        skew_expect = full.search_fixed(np.tile(qbs[r][:m], nq // 10), m, algo="plain")
        assert np.array_equal(sk.astype(np.uint64), skew_expect), r
        assert raised, r


def _key(t, pos, p):
    """p-char zero-padded key of suffix pos as an integer (the prefix table's key)."""
    k = 0
    for j in range(p):
        k = 4 * k + (int(t[pos + j]) if pos + j < len(t) else 0)
    return k


@pytest.mark.parametrize("inl,p", [(0, 10), (1, 9), (2, 10), (2, 12), (4, 10)])
def test_part_prefix_table_key_interval(sas, inl, p):
    """A part's prefix table covers only its own key interval (its first suffix's p-char key
    .. its last one's, + two entries of rank sa_n): stats name the interval, the table is
    that many entries, and PREFIX on the part equals PLAIN on the part for queries inside,
    below and above the interval (clamped lookups), at m below, at and above p; occurrence
    ranges equal the whole index's clipped to the part's ranks, inline slots or not."""
    import torch
    from sas_amd import _lib
    n, W = 2_000_003, 4
    t = sas.random_string(n, seed=91)
    dt = torch.from_numpy(t).cuda()
    whole = sas.SaNaive.build(t, lcp=False, stree=False, sector=False, llcp=False, prefix=p, prefix_inline=2)
    rng = np.random.default_rng(inl * 31 + p)
    for g in range(W):
        part = sas.SaNaive.build_part(dt, g, W, lcp=False, stree=False, sector=False, llcp=False, prefix=p,
                                      prefix_inline=inl)
        st = part.stats()
        sa = part.suffix_array()
        k0, k1 = _key(t, int(sa[0]), p), _key(t, int(sa[-1]), p)
        assert st["prefix_key_lo"] == k0 and st["prefix_entries"] == k1 - k0 + 3, (g, st)
        w = 16 * inl if inl else 5
        assert st["prefix_bytes"] == st["prefix_entries"] * w
        assert st["prefix_entries"] < (4 ** p) // 2, g  # an interval, not the key space
        for m in (p - 3, p, 32):
            offs = rng.integers(0, n - m, 6000)
            qs = np.stack([t[o:o + m] for o in offs])
            qs[:1000] = rng.integers(0, 4, (1000, m))  # misses, most outside this part's keys
            qs[1000] = 0
            qs[1001] = 3
            # just below / at / above the part's first and last keys
            for j, pos in enumerate((int(sa[0]), int(sa[-1]))):
                base = np.array([t[pos + c] if pos + c < n else 0 for c in range(m)], np.uint8)
                qs[1002 + 4 * j] = base
                lo = base.copy()
                lo[min(p, m) - 1] = max(int(lo[min(p, m) - 1]) - 1, 0)
                qs[1003 + 4 * j] = lo
                hi = base.copy()
                hi[min(p, m) - 1] = min(int(hi[min(p, m) - 1]) + 1, 3)
                qs[1004 + 4 * j] = hi
                qs[1005 + 4 * j] = np.where(np.arange(m) < min(p, m), base, 3)
            qb = qs.reshape(-1).copy()
            plain = part.search_fixed(qb, m, algo="plain")
            assert np.array_equal(part.search_fixed(qb, m, algo="prefix"), plain), (g, m)
            if inl == 2 and m <= 32:
                words = sas.SaNaive.pack_queries(torch.from_numpy(qb).cuda(), m)
                got = part.search_packed(words, m)
                torch.cuda.synchronize()
                assert np.array_equal(got.cpu().numpy().astype(np.uint64), plain), (g, m)
            dq = torch.from_numpy(qb).cuda()
            lo, hi = part.search_range_fixed(dq, m)
            wl, wh = whole.search_range_fixed(dq, m)
            r0, r1 = part.rank_lo, part.rank_lo + part.sa_n
            torch.cuda.synchronize()
            assert np.array_equal(lo.cpu().numpy(), np.clip(wl.cpu().numpy(), r0, r1)), (g, m)
            assert np.array_equal(hi.cpu().numpy(), np.clip(wh.cpu().numpy(), r0, r1)), (g, m)
            if inl >= 2:
                lo2, hi2 = part.search_range_fixed(dq, m, flags=_lib.SAS_RANGE_NO_INLINE)
                torch.cuda.synchronize()
                assert torch.equal(lo, lo2) and torch.equal(hi, hi2), (g, m)
        part.free()


@pytest.mark.timeout(600)
def test_two_slot_table_ranks_above_2e32(sas):
    """A one-part index (sas_build_part_gen, parts = 1: the whole table) of a 1.125 x 2^32-char
    text holds more than 2^32 suffixes: the two-suffix inline table carries bits 32..39 of
    each entry's rank in slot 1's rank word, so PREFIX (bytes and packed words) equals PLAIN
    and the inline-slot ranges equal the bisection's, with lower bounds past rank 2^32."""
    import torch
    from sas_amd import _lib
    n, m, seed = 9 << 29, 32, 57
    part = sas.SaNaive.build_part_gen(n, seed=seed, part=0, parts=1, lcp=False, stree=False, sector=False,
                                      llcp=False, quad=True, prefix=15, prefix_inline=2, top2_levels=15)
    st = part.stats()
    assert st["sa_entries"] == n and st["prefix_entries"] == 4 ** 15 + 1 and st["prefix_key_lo"] == 0
    rng = np.random.default_rng(5)
    nq = 400_000
    off = torch.from_numpy(rng.integers(0, n - m, nq).astype(np.int64)).cuda()
    q = torch.empty(nq * m, dtype=torch.uint8, device="cuda")
    part.extract(off, torch.full((nq,), m, dtype=torch.int32, device="cuda"),
                 torch.arange(nq, device="cuda", dtype=torch.int64) * m, q)
    q[: 20_000 * m] = torch.from_numpy(rng.integers(0, 4, 20_000 * m, dtype=np.uint8)).cuda()  # misses
    # the last ~1/9 of the ranks lie past 2^32: queries starting with 3s land there
    q[20_000 * m: 60_000 * m].view(40_000, m)[:, :3] = 3
    plain = part.search_fixed(q, m, algo="plain")
    pre = part.search_fixed(q, m, algo="prefix")
    pk = part.search_packed(sas.SaNaive.pack_queries(q, m), m)
    lo, hi = part.search_range_fixed(q, m)
    lo2, hi2 = part.search_range_fixed(q, m, flags=_lib.SAS_RANGE_NO_INLINE)
    torch.cuda.synchronize()
    assert torch.equal(plain, pre) and torch.equal(plain, pk)
    assert torch.equal(lo, lo2) and torch.equal(hi, hi2)
    assert int((lo >= (1 << 32)).sum().item()) > nq // 20
    part.free()


def test_inline_tables_on_40bit_sa(sas):
    """The one/two/four-suffix inline prefix tables beside a packed 40-bit SA (allowed while
    n < 2^32: ranks and positions fit the entries' 32-bit fields) give the u32 index's
    PREFIX positions, probes and ranges; routing words packed by sas_route_pack equal
    sas_pack_queries'."""
    import torch
    n, m = 500_009, 32
    t = sas.random_string(n, seed=31)
    qb = queries(t, 20_000, m, 4)
    ref = sas.SaNaive.build(t, prefix=10, prefix_inline=2)
    exp, epr = ref.search_fixed(qb, m, algo="prefix", probes=True)
    assert np.array_equal(exp, ref.search_fixed(qb, m, algo="plain"))
    for inl in (1, 2, 4):
        idx = sas.SaNaive.build(t, sa40=True, prefix=10, prefix_inline=inl)
        assert idx.stats()["sa_width"] == 5
        got, pr = idx.search_fixed(qb, m, algo="prefix", probes=True)
        assert np.array_equal(got, exp), inl
        if inl == 2:
            assert np.array_equal(pr, epr)
    dq = torch.from_numpy(qb).cuda()
    _, words, slot = ref.route_pack(torch.empty(0, dtype=torch.int64, device="cuda"), dq, m, cap=len(qb) // m,
                                    packed=True)
    w2 = sas.SaNaive.pack_queries(dq, m)
    torch.cuda.synchronize()
    assert np.array_equal(words.cpu().numpy()[slot.cpu().numpy()], w2.cpu().numpy())


def test_route_pack_argument_errors(sas):
    """sas_route_pack_cap: cap = 0 and SAS_ROUTE_PACKED with m > 32 are EINVAL."""
    import torch
    from sas_amd import _lib
    from sas_amd._lib import SasError
    t = sas.random_string(10_007, seed=2)
    idx = sas.SaNaive.build(t)
    q = torch.from_numpy(np.concatenate([t[:40], t[100:140]])).cuda()
    sp = torch.empty(0, dtype=torch.int64, device="cuda")
    with pytest.raises(SasError):
        idx.route_pack(sp, q, 40, cap=2, packed=True)  # m > 32
    counts = torch.empty(1, dtype=torch.int64, device="cuda")
    send = torch.empty(80, dtype=torch.uint8, device="cuda")
    slot = torch.empty(2, dtype=torch.int64, device="cuda")
    rc = _lib.lib().sas_route_pack_cap(idx._h, None, 0, q.data_ptr(), 40, 2, 0, counts.data_ptr(), send.data_ptr(),
                                       slot.data_ptr(), None, _lib.SAS_DEVICE_PTRS)
    assert rc != 0
    c, s2, sl = idx.route_pack(sp, q, 40, cap=2)
    torch.cuda.synchronize()
    assert c.tolist() == [2] and sorted(sl.tolist()) == [0, 1]
    assert torch.equal(s2.view(2, 40)[sl], q.view(2, 40))


def test_route_pack_cap_one_pass_and_gather(sas):
    """sas_route_pack_cap (one pass: wave-aggregated bucket ranks, one global claim per
    block and bucket) with W = 5 parts, byte and packed slots: counts = the histogram of
    sas_route, every query inside its bucket's slots, slots distinct, bytes / words at
    their slot; a cap below a bucket's count clamps the overflow to the last slot, and
    sas_shard_gather puts positions back in query order and raises the overflow flag."""
    import torch
    n, W = 300_007, 5
    t = sas.random_string(n, seed=61)
    idxs = [sas.SaNaive.build_part(t, g, W, lcp=False, stree=False, sector=False) for g in range(W)]
    splitters = torch.tensor([int(ix.suffix_array(1)[0]) for ix in idxs[1:]], dtype=torch.int64).cuda()
    rng = np.random.default_rng(8)
    for m, packed in ((24, False), (32, False), (32, True), (13, True)):
        offs = rng.integers(0, n - m, 30_011)
        qb = np.concatenate([t[o:o + m] for o in offs] + [rng.integers(0, 4, 7001 * m, dtype=np.uint8)])
        nq = len(qb) // m
        dq = torch.from_numpy(qb).cuda()
        dest = idxs[0].route(splitters, dq, m).cpu().numpy().astype(np.int64)
        hist = np.bincount(dest, minlength=W)
        cap = int(hist.max()) + 3
        counts, send, slot = idxs[0].route_pack(splitters, dq, m, cap=cap, packed=packed)
        c, s, sl = counts.cpu().numpy(), send.cpu().numpy(), slot.cpu().numpy()
        assert c.tolist() == hist.tolist(), (m, packed)
        assert len(np.unique(sl)) == nq
        assert ((sl >= dest * cap) & (sl < dest * cap + hist[dest])).all()
        if packed:
            words = sas.SaNaive.pack_queries(dq, m).cpu().numpy()
            assert np.array_equal(s.view(np.uint64)[sl], words.view(np.uint64))
        else:
            assert np.array_equal(s.reshape(W * cap, m)[sl], qb.reshape(nq, m))
        # gather: "positions" = the slot numbers themselves come back as the query index
        back = torch.full((W * cap,), -1, dtype=torch.int64, device="cuda")
        back[slot] = torch.arange(nq, device="cuda")
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        got = idxs[0].shard_gather(back, slot, counts=counts, cap=cap, overflow=flag)
        assert np.array_equal(got.cpu().numpy(), np.arange(nq)) and int(flag.item()) == 0
        # overflow: the largest bucket gets 7 fewer slots than it needs
        small = int(hist.max()) - 7
        counts, send, slot = idxs[0].route_pack(splitters, dq, m, cap=small, packed=packed)
        sl = slot.cpu().numpy()
        big = hist > small
        assert counts.cpu().numpy().tolist() == hist.tolist()
        clamped = sl == W * small - 1
        assert int(clamped.sum()) >= int((hist[big] - small).sum())
        ok = ~np.isin(dest, np.nonzero(big)[0])
        assert ((sl[ok] >= dest[ok] * small) & (sl[ok] < dest[ok] * small + hist[dest[ok]])).all()
        idxs[0].shard_gather(torch.zeros(W * small, dtype=torch.int64, device="cuda"), slot, counts=counts, cap=small,
                             overflow=flag)
        assert int(flag.item()) == 1, (m, packed)


def test_inline_slots_above_2e32(sas):
    """A part index of a 1.5 x 2^32-char text (local ranks < 2^32, positions up to 33 bits)
    carries the two- and four-suffix inline tables with bits 32..39 of each slot's SA value
    in slot 1: PREFIX (bytes and packed words) equals PLAIN on the same part, and the
    inline-slot ranges equal the bisection's; part of the answers lie past 2^32."""
    import torch
    from sas_amd import _lib
    n, m, W, g = 3 << 31, 32, 4, 3
    t = sas.random_string(n, seed=41, device="cuda")
    rng = np.random.default_rng(6)
    nq = 400_000
    off = torch.from_numpy(rng.integers(0, n - m, nq)).cuda()
    ar = torch.arange(m, device="cuda")
    q = t[(off[:, None] + ar[None, :]).reshape(-1)].contiguous()
    q[: 20_000 * m] = torch.from_numpy(rng.integers(0, 4, 20_000 * m, dtype=np.uint8)).cuda()  # misses
    for inl in (2, 4):
        part = sas.SaNaive.build_part(t, g, W, lcp=False, stree=False, sector=False, llcp=False, prefix=15,
                                      prefix_inline=inl)
        plain = part.search_fixed(q, m, algo="plain")
        pre = part.search_fixed(q, m, algo="prefix")
        pk = part.search_packed(sas.SaNaive.pack_queries(q, m), m)
        torch.cuda.synchronize()
        assert torch.equal(plain, pre) and torch.equal(plain, pk), inl
        # a quarter of the lower bounds lie in this part, a third of those past 2^32
        assert int((plain >= (1 << 32)).sum().item()) > nq // 20
        lo, hi = part.search_range_fixed(q, m)
        lo2, hi2 = part.search_range_fixed(q, m, flags=_lib.SAS_RANGE_NO_INLINE)
        torch.cuda.synchronize()
        assert torch.equal(lo, lo2) and torch.equal(hi, hi2), inl
        part.free()


def test_build_gen_equals_byte_build(sas):
    """sas_build_gen / sas_build_part_gen generate random_string(n, seed) on the GPU straight
    into the packed text: the text (read back through sas_extract), the SA and the part
    ranges equal those of the same index built from sas_gen_text's bytes, for an n that is
    not a multiple of the 32-char word, and the searches agree."""
    import torch
    n, seed, W = 3_000_017, 77, 3
    t = sas.random_string(n, seed=seed)
    a = sas.SaNaive.build(t, lcp=False, stree=False, sector=False, llcp=False, prefix=10, prefix_inline=2)
    b = sas.SaNaive.build_gen(n, seed=seed, lcp=False, stree=False, sector=False, llcp=False, prefix=10,
                              prefix_inline=2)
    assert np.array_equal(a.suffix_array(), b.suffix_array())
    got = torch.empty(n, dtype=torch.uint8, device="cuda")
    b.extract(torch.zeros(1, dtype=torch.int64, device="cuda"), torch.tensor([n], dtype=torch.int32, device="cuda"),
              torch.zeros(1, dtype=torch.int64, device="cuda"), got)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), t)
    qb = queries(t, 20_000, 32, 3)
    assert np.array_equal(a.search_fixed(qb, 32, algo="prefix"), b.search_fixed(qb, 32, algo="prefix"))
    dt = torch.from_numpy(t).cuda()
    for g in range(W):
        p = sas.SaNaive.build_part(dt, g, W, lcp=False, stree=False, sector=False, llcp=False, prefix=10,
                                   prefix_inline=2)
        q = sas.SaNaive.build_part_gen(n, seed=seed, part=g, parts=W, lcp=False, stree=False, sector=False,
                                       llcp=False, prefix=10, prefix_inline=2)
        assert (p.rank_lo, p.sa_n, p.next_pos) == (q.rank_lo, q.sa_n, q.next_pos), g
        assert np.array_equal(p.suffix_array(), q.suffix_array()), g
        p.free()
        q.free()


@pytest.mark.timeout(600)
def test_c4_shape_w8_loopback_past_2e32(sas):
    """configs[4]'s step at W = 8 on one GPU (loopback exchange, one thread per rank) over a
    2^32-char text: each rank's part from sas_build_part_gen (generated packed text, 40-bit
    SA, fused quad leaves, two-suffix inline table at the bench's p = 16, each part's table
    sized to its own key interval: about 1/8 of the 4^16 keys, so eight parts fit one GPU),
    PREFIX queries crossing as 8-B words into fixed-capacity buckets (max_nq, check=False +
    assert_no_overflow), positions equal to the whole index's PLAIN search, and the bench's
    per-rank lower-bound proof (bench.c4_proof) on every rank."""
    import torch
    import bench
    from sas_amd.shard import ShardedSearch
    n, W, m, nq, seed = 1 << 32, 8, 32, 200_000, 4242
    whole = sas.SaNaive.build_gen(n, seed=seed, lcp=False, stree=False, sector=False, quad=False, llcp=False,
                                  prefix=False)
    qbs, expect = [], []
    for r in range(W):
        off = torch.from_numpy(bench.rank_query_offsets(n, nq, m, r).astype(np.int64)).cuda()
        q = torch.empty(nq * m, dtype=torch.uint8, device="cuda")
        whole.extract(off, torch.full((nq,), m, dtype=torch.int32, device="cuda"),
                      torch.arange(nq, device="cuda", dtype=torch.int64) * m, q)
        q[: 1000 * m] = torch.from_numpy(np.random.default_rng(r).integers(0, 4, 1000 * m, dtype=np.uint8)).cuda()
        qbs.append(q)
        expect.append(whole.search_fixed(q, m, algo="plain"))
    torch.cuda.synchronize()
    whole.free()
    torch.cuda.empty_cache()
    parts = [sas.SaNaive.build_part_gen(n, seed=seed, part=g, parts=W, lcp=False, stree=False, sector=False,
                                        quad=True, llcp=False, prefix=16, prefix_inline=2, top2_levels=15)
             for g in range(W)]
    assert sum(p.sa_n for p in parts) == n
    ents = [p.stats()["prefix_entries"] for p in parts]
    # contiguous key intervals: every key once, plus the 2 sentinel entries and the shared
    # boundary keys of adjacent parts
    assert 0.99 * 4 ** 16 <= sum(ents) <= 4 ** 16 + 2 * W and max(ents) < 1.1 * 4 ** 16 / W, ents
    assert max(p.next_pos for p in parts) == n or parts[-1].next_pos == n
    lb = Loopback(W)
    res, errs = {}, []

    def rank_main(r):
        try:
            d = lb.rank(r)
            eng = ShardedSearch(parts[r], d, W, r, torch.device("cuda"), algo="prefix", max_nq=nq)
            assert eng.packed(m) and eng.bucket_lookup(m)
            out = torch.empty(nq, dtype=torch.int64, device="cuda")
            eng.search_fixed(qbs[r], m, check=False, out=out)
            eng.assert_no_overflow()
            torch.cuda.synchronize()
            pr = bench.c4_proof(torch, parts[r], eng, n, m, W, r, 200)
            res[r] = (out.cpu().numpy(), pr)
        except Exception as e:  # surfaced below
            errs.append((r, repr(e)))
            lb.bar.abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(W)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    assert not errs, errs
    for r in range(W):
        out, pr = res[r]
        assert np.array_equal(out, expect[r].cpu().numpy()), r
        assert pr["checked"] > 0 and pr["failures"] == 0, (r, pr)
    assert sum(int((e >= (1 << 32) - (1 << 30)).sum().item()) for e in expect) > 0
    for p in parts:
        p.free()
