"""world_size-2 gloo test of the multi-GPU harness (bench.py) on the CPU:
per-rank query shards, barrier-bracketed timing, MAX-over-ranks reduction, and
that the shards' answers equal a single process's answers (replicated index,
no data-path collective)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import bench
from oracle import pyoracle as O


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, ws, port, res):
    import time
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    n, nq, m = 1 << 14, 512, 24
    t = O.random_string(n)
    sa = O.build_sa(t)
    tp = O.padded(t)
    off = bench.rank_query_offsets(n, nq, m, rank)
    qb = np.concatenate([t[o:o + m] for o in off.astype(np.int64)] + [np.zeros(64, np.uint8)])
    out = {}

    def step():
        out["pos"], _ = O.search_many(tp, n, sa, qb, np.arange(nq, dtype=np.uint64) * m,
                                      np.full(nq, m, np.uint32), "binary_search", 1)
        if rank == 1:
            time.sleep(0.02)  # uneven ranks: the MAX must be the slow one

    def reduce_max(x):
        tt = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    el = bench.timed_loop(step, 3, 1, lambda: None, dist.barrier, reduce_max)
    res[rank] = (el, off.tolist(), out["pos"].tolist())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 8])
def test_rank_harness(ws):
    """world_size 2, and 8 (the driver's largest scaling run) rehearsed with gloo."""
    mgr = mp.Manager()
    res = mgr.dict()
    mp.spawn(worker, args=(ws, free_port(), res), nprocs=ws, join=True)
    els = [res[r][0] for r in range(ws)]
    assert len(set(els)) == 1 and els[0] >= 3 * 0.02  # every rank reports the same MAX
    offs = [tuple(res[r][1]) for r in range(ws)]
    assert len(set(offs)) == ws  # disjoint query streams per rank
    # replicated index: each shard's answers equal a single-process search of those queries
    n, m = 1 << 14, 24
    t = O.random_string(n)
    sa = O.build_sa(t)
    tp = O.padded(t)
    for off, pos in ((res[r][1], res[r][2]) for r in range(ws)):
        for o, p in zip(off[:50], pos[:50]):
            assert O.search_one(tp, n, sa, t[o:o + m])[0] == p
            assert list(t[p:p + m]) == list(t[o:o + m])


# ------------------------------------------------------------------ sharded-text mode
class OracleShard:
    """CPU stand-in for a GPU shard index (same interface as sas_amd.SaNaive)
    so the all-to-all exchange of sas_amd.shard.ShardedSearch runs on gloo."""

    def __init__(self, t, sa_full, lo, hi):
        self.tb = bytes(t.tolist())
        self.n = len(t)
        self.sa = sa_full[lo:hi]
        self.next = int(sa_full[hi]) if hi < self.n else self.n
        self.searched = 0  # slots searched by search_buckets

    def suffix_array(self, count):
        return self.sa[:count]

    def route(self, splitters, qbytes, m):
        import torch
        sp = [int(s) for s in splitters.tolist()]
        qs = qbytes.view(-1, m).tolist()
        return torch.tensor([sum(self.tb[s:] < bytes(q) for s in sp) for q in qs], dtype=torch.int32)

    def route_pack(self, splitters, qbytes, m, cap=None, send=None):
        """sas_route_pack / sas_route_pack_cap semantics in torch: queries grouped by
        destination; with cap, bucket w owns send slots [w*cap, (w+1)*cap) and a query past
        its bucket's cap is dropped (slot W*cap - 1, counts > cap)."""
        import torch
        nq = qbytes.numel() // m
        W = splitters.numel() + 1
        dest = self.route(splitters, qbytes, m).to(torch.int64)
        counts = torch.bincount(dest, minlength=W)
        order = torch.argsort(dest, stable=True)
        starts = torch.cumsum(counts, 0) - counts
        rank_in = torch.empty(nq, dtype=torch.int64)
        rank_in[order] = torch.arange(nq) - starts[dest[order]]
        if not cap:
            slot = starts[dest] + rank_in
            qsend = torch.zeros(nq * m, dtype=torch.uint8)
            qsend.view(nq, m)[slot] = qbytes.view(nq, m)
            return counts, qsend, slot
        if send is None or send.numel() < W * cap * m:
            send = torch.zeros(W * cap * m, dtype=torch.uint8)
        ok = rank_in < cap
        slot = torch.where(ok, dest * cap + rank_in, torch.full_like(dest, W * cap - 1))
        send.view(-1, m)[slot[ok]] = qbytes.view(nq, m)[ok]
        return counts, send[: W * cap * m], slot

    def shard_gather(self, back, slot, out=None, counts=None, cap=0, overflow=None):
        """sas_shard_gather semantics: out[k] = back[slot[k]]; overflow raised (never
        cleared) when a bucket's count passed cap."""
        import torch
        res = back[slot]
        if overflow is not None and bool((counts > cap).any()):
            overflow.fill_(1)
        if out is None:
            return res
        out.copy_(res)
        return out

    def search_buckets(self, recv, m, cap, counts, algo=None, out=None):
        """sas_search_buckets semantics: only the first counts[b] slots of bucket b are
        searched and written; the rest of `out` is left alone.  Counts the lookups."""
        import torch
        if out is None:
            out = torch.full((counts.numel() * cap,), -1, dtype=torch.int64)
        for b, c in enumerate(counts.tolist()):
            c = min(int(c), cap)
            if c:
                out[b * cap:b * cap + c] = self._search(recv[b * cap * m:(b * cap + c) * m], m)
            self.searched += c
        return out

    def search_fixed(self, qbytes, m, algo=None, out=None):
        import torch
        res = self._search(qbytes, m)
        if out is not None:
            out.copy_(res)
            return out
        return res

    def _search(self, qbytes, m):
        import torch
        out = []
        for q in qbytes.view(-1, m).tolist():
            q = bytes(q)
            l, r = 0, len(self.sa)
            while l < r:
                mid = (l + r) // 2
                if self.tb[int(self.sa[mid]):] < q:
                    l = mid + 1
                else:
                    r = mid
            out.append(int(self.sa[l]) if l < len(self.sa) else self.next)
        return torch.tensor(out, dtype=torch.int64)


def shard_worker(rank, ws, port, res):
    import torch
    import torch.distributed as dist
    from sas_amd.shard import ShardedSearch, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    n, nq, m = 3000, 200, 12
    t = O.random_string(n, seed=5)
    sa = O.build_sa(t)
    lo, hi = shard_range(n, ws, rank)
    eng = ShardedSearch(OracleShard(t, sa, lo, hi), dist, ws, rank, "cpu")
    rng = np.random.default_rng(rank)
    offs = rng.integers(0, n - m, nq)
    qs = np.stack([t[o:o + m] for o in offs])
    qs[: nq // 4] = rng.integers(0, 4, (nq // 4, m))  # negatives too
    qs[-1] = 3  # above every suffix -> n
    dq = torch.from_numpy(qs.reshape(-1).copy())
    pos = eng.search_fixed(dq, m)  # fixed-capacity buckets, the overflow flag checked
    pos2 = eng.search_fixed(dq, m, check=False)  # deferred check
    eng.assert_no_overflow()
    exact = eng.search_fixed_exact(dq, m)  # variable-size exchanges
    assert pos.tolist() == pos2.tolist() == exact.tolist()
    # the pipelined step: three pieces, async exchanges overlapped with the other pieces' work
    pipe = ShardedSearch(OracleShard(t, sa, lo, hi), dist, ws, rank, "cpu", chunks=3)
    assert pipe.search_fixed(dq, m).tolist() == exact.tolist()
    out = torch.full((nq,), -1, dtype=torch.int64)
    pipe.search_fixed(dq, m, check=False, out=out)
    pipe.assert_no_overflow()
    assert out.tolist() == exact.tolist()
    # skewed batch (every query the same) into tiny buckets: the checked step overflows and
    # redoes itself exactly; the deferred one reports the overflow
    tight = ShardedSearch(OracleShard(t, sa, lo, hi), dist, ws, rank, "cpu", slack=0.5, min_cap=0)
    skew = torch.from_numpy(np.tile(qs[nq // 2], nq // 4).copy())
    got = tight.search_fixed(skew, m)
    assert got.tolist() == eng.search_fixed_exact(skew, m).tolist()
    tight.search_fixed(skew, m, check=False)
    with pytest.raises(RuntimeError):
        tight.assert_no_overflow()
    tight3 = ShardedSearch(OracleShard(t, sa, lo, hi), dist, ws, rank, "cpu", slack=0.5, min_cap=0, chunks=3)
    assert tight3.search_fixed(skew, m).tolist() == got.tolist()  # overflow redone exactly
    tight3.search_fixed(skew, m, check=False)
    with pytest.raises(RuntimeError):
        tight3.assert_no_overflow()
    # the bounded lookup: the ranks together search exactly the queries they were given (not
    # W * cap slots each); ranks pass different batch sizes, and change them between steps,
    # with the per-step capacity agreement and with a declared max_nq
    for mx in (None, nq):
        shard = OracleShard(t, sa, lo, hi)
        eng2 = ShardedSearch(shard, dist, ws, rank, "cpu", algo="plain", max_nq=mx)
        total = 0
        for step in range(3):
            k = nq - 17 * ((rank + step) % 3)  # differs across ranks and steps
            got = eng2.search_fixed(dq[:k * m], m)
            assert got.tolist() == exact.tolist()[:k]
            total += k
        both = torch.tensor([shard.searched, total], dtype=torch.int64)
        dist.all_reduce(both)
        assert both[0] == both[1], (int(both[0]), int(both[1]))
    # a batch past the declared max_nq is not refused on one rank (the others would hang in
    # the exchange): it runs with the agreed capacity, and a bucket it overfills is redone
    # exactly by the step every rank agrees on
    for mc in (256, 0):
        big = ShardedSearch(OracleShard(t, sa, lo, hi), dist, ws, rank, "cpu", algo="plain", max_nq=10, min_cap=mc)
        assert big.search_fixed(dq, m).tolist() == exact.tolist()
    # STREE (the constructor's default) has no bounded lookup: every slot is searched
    dflt = ShardedSearch(OracleShard(t, sa, lo, hi), dist, ws, rank, "cpu")
    assert dflt.algo == "stree" and not dflt.bucket_lookup(m)
    assert dflt.search_fixed(dq, m).tolist() == exact.tolist()
    res[rank] = (qs.tolist(), pos.tolist())
    dist.destroy_process_group()


@pytest.mark.parametrize("ws", [3, 8])
def test_sharded_exchange(ws):
    mgr = mp.Manager()
    res = mgr.dict()
    mp.spawn(shard_worker, args=(ws, free_port(), res), nprocs=ws, join=True)
    n = 3000
    t = O.random_string(n, seed=5)
    sa = O.build_sa(t)
    tp = O.padded(t)
    for r in range(ws):
        qs, pos = res[r]
        for q, p in zip(qs, pos):
            assert O.search_one(tp, n, sa, np.array(q, np.uint8))[0] == p
