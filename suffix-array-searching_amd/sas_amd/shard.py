"""Sharded-text mode: the suffix array is split into SA-rank ranges,
one per GPU; queries are routed to the GPU owning their lower bound and the
positions come back -- the only place this engine uses a collective.

    rank g holds global SA ranks [g*n/W, (g+1)*n/W) (SaNaive.build(rank_range=...) or
    SaNaive.build_part), splitters = text positions of the first suffix of shards 1..W-1
    (all-gathered once),
    step: route + group by destination into fixed-capacity buckets (sas_route_pack_cap)
          -> all_to_all query bytes (equal splits; PREFIX with m <= 32: 8-B packed words)
          -> local lookup of every received slot -> all_to_all positions back (equal splits)
          -> gather by send slot.

Hash-partitioning the SA would break its order (a lower bound would need every
shard); rank ranges keep each answer on exactly one shard.  The collective is
`torch.distributed.all_to_all_single` (RCCL over xGMI with backend "nccl";
gloo in the CPU tests).  Payload per query: m bytes out, 8 bytes back.

Fixed-capacity buckets (cap = nq * slack / W per destination, agreed by all ranks) make
both exchanges equal-split, so a step issues no host synchronisation: no .tolist(), no
.item().  The per-bucket counts cross in a W-element all-to-all beside the queries, and the
local lookup searches only the filled slots of each received bucket (sas_search_buckets),
so the ranks together search exactly the queries they were given, not W * cap slots each.
A bucket that overflows its cap is detected on the device; with `check=True` (the default)
the step reads that one flag and redoes itself with exact variable-size exchanges, so
results are always exact; `check=False` defers the flag to `assert_no_overflow()` (the
bench calls it once after its timed loop).

The capacity is agreed by a collective that every rank runs: once, in the constructor, for
a declared `max_nq` (steps of at most that many queries then run no extra collective), or
at the start of every step otherwise.  Ranks may pass different batch sizes either way.

At world size 1 every query is the rank's own: the exchanges are the identity, and so are the
route (one bucket) and the gather (slot = query index), so the step is the local lookup of the
query batch itself (round 6: 0.49 -> ~0.31 ms per 10^7 at n = 2^32).  `routed=True` keeps the
route + identity exchange + gather shape (what each rank of a W > 1 step runs), and
`exchange_self=True` also sends the exchanges through the process group, which is how the
world-1 RCCL test exercises the exchange path.
"""
from __future__ import annotations


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Global SA ranks owned by `rank`: contiguous and balanced."""
    return (n * rank) // world, (n * (rank + 1)) // world


class ShardedSearch:
    """`index` needs: .route(splitters, qbytes, m) -> dest shard per query,
    .search_fixed(qbytes, m, algo=...) -> positions (int64), .suffix_array(1) ->
    its first SA value; the GPU implementation (sas_amd.SaNaive) also has
    .route_pack(splitters, qbytes, m, cap=None) (the fused send side),
    .search_buckets(recv, m, cap, counts, algo=...) (the bounded local lookup) and
    .shard_gather(back, slot, ...) (the receive side)."""

    SLACK = 1.125  # bucket capacity over the balanced share

    def __init__(self, index, dist, world: int, rank: int, device, algo: str = "stree", group=None,
                 slack: float | None = None, min_cap: int = 256, chunks: int = 1, max_nq: int | None = None,
                 exchange_self: bool = False, routed: bool = False):
        """chunks > 1: a step cuts its batch into that many pieces and overlaps one piece's
        exchanges (all_to_all_single with async_op, on the collective's own stream) with
        another's routing, lookup and gather.  Every rank must use the same value.
        max_nq: the largest batch any step of this rank will pass; the bucket capacity is then
        agreed here, once (a collective every rank runs), and steps add none.  Without it every
        step agrees on its capacity first (one all_reduce and a host read per step)."""
        import torch
        self.chunks = max(1, int(chunks))
        self.index, self.dist, self.world, self.rank = index, dist, world, rank
        self.device, self.algo, self.group = device, algo, group
        self.slack = self.SLACK if slack is None else slack
        self.min_cap = min_cap
        self.exchange = world > 1 or exchange_self
        # world 1 without exchange: route and gather are the identity too (routed=False)
        self.identity = not self.exchange and not routed
        self._sa_width = index.stats().get("sa_width", 4) if hasattr(index, "stats") else 4
        first = torch.tensor([int(index.suffix_array(1)[0])], dtype=torch.int64, device=device)
        firsts = [torch.empty_like(first) for _ in range(world)]
        dist.all_gather(firsts, first, group=group)
        # first suffix of shards 1..W-1, in increasing suffix order
        self.splitters = torch.cat(firsts[1:]).to(torch.int64) if world > 1 else torch.empty(0, dtype=torch.int64,
                                                                                              device=device)
        self._bufs = {}
        self.overflow = torch.zeros(1, dtype=torch.int32, device=device)
        self.max_nq = None if max_nq is None else int(max_nq)
        self._cap_fixed = None
        if self.max_nq is not None:
            self._cap_fixed = self._agree(self._local_cap(-(-self.max_nq // self.chunks)))

    # ---------------------------------------------------------------- capacity
    def _local_cap(self, nq: int) -> int:
        if self.world == 1:
            return max(nq, 1)
        return max(1, min(nq, int(nq * self.slack / self.world) + self.min_cap))

    def _agree(self, cap: int) -> int:
        """MAX over ranks (a collective: every rank calls it at the same point)."""
        import torch
        t = torch.tensor([cap], dtype=torch.int64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def capacity(self, nq: int) -> int:
        """Per-destination bucket capacity for a piece of nq queries: every rank must use the
        same one (equal all-to-all splits).  With max_nq it is the constructor's agreed value
        (no collective); otherwise the MAX over ranks of each rank's own need, agreed now --
        every rank runs this collective at the start of every step, whatever its nq."""
        if self._cap_fixed is not None:
            # a piece larger than max_nq declared is not refused here: raising on one rank
            # would leave the others blocked in the exchange.  It runs with the agreed
            # capacity; a bucket it overfills raises the device overflow flag, which every
            # rank sees (check=True redoes the step with exact exchanges, check=False fails
            # in assert_no_overflow on every rank)
            return self._cap_fixed
        return self._agree(self._local_cap(nq))

    def packed(self, m: int) -> bool:
        """Queries cross the exchange as 8-B 2-bit words (SAS_ROUTE_PACKED) when the local
        lookup takes them: PREFIX, m <= 32 (4x less all-to-all traffic at m = 32)."""
        return self.algo == "prefix" and m <= 32 and hasattr(self.index, "search_packed")

    def _buffers(self, m: int, cap: int, piece: int = 0):
        import torch
        key = (m, cap, piece)
        if key not in self._bufs:
            W = self.world
            if self.packed(m):
                q = {"send": torch.zeros(W * cap, dtype=torch.int64, device=self.device),
                     "recv": torch.zeros(W * cap, dtype=torch.int64, device=self.device)}
            else:
                q = {"send": torch.zeros(W * cap * m, dtype=torch.uint8, device=self.device),
                     "recv": torch.zeros(W * cap * m, dtype=torch.uint8, device=self.device)}
            self._bufs[key] = dict(q, back=torch.empty(W * cap, dtype=torch.int64, device=self.device),
                                   local=torch.empty(W * cap, dtype=torch.int64, device=self.device),
                                   rcounts=torch.empty(W, dtype=torch.int64, device=self.device))
        return self._bufs[key]

    # ---------------------------------------------------------------- steps
    def _forward(self, buf, send, counts, async_op=False):
        """Queries (and their per-bucket counts) to their owners.  Returns the received
        slots, the received counts and the pending works."""
        if not self.exchange:  # world 1: the exchange is the identity
            return send, counts, []
        w1 = self.dist.all_to_all_single(buf["rcounts"], counts, group=self.group, async_op=async_op)
        w2 = self.dist.all_to_all_single(buf["recv"], send, group=self.group, async_op=async_op)
        return buf["recv"], buf["rcounts"], [w for w in (w1, w2) if w is not None]

    # the algorithms sas_search_buckets takes (csrc/sas_search.hip, sas_search_buckets):
    # PLAIN / LCP / LLCP / PREFIX, and QUAD for m <= 32
    BUCKET_ALGOS = ("plain", "lcp", "llcp", "prefix")

    def bucket_lookup(self, m: int) -> bool:
        """The bounded lookup (only the filled slots) applies to this algo and m."""
        if not hasattr(self.index, "search_buckets") or self._sa_width == 8:
            return False
        return self.packed(m) or self.algo in self.BUCKET_ALGOS or (self.algo == "quad" and m <= 32)

    def _lookup(self, buf, recv, rcounts, m: int, cap: int):
        """The local lookup of the filled received slots (positions into buf["local"]).
        Algorithms without a bounded lookup (STREE, SECTOR, INLINE, INTERP, QUAD past 32
        chars) search every slot: an unfilled slot holds zero bytes (a valid query whose
        answer nobody gathers)."""
        pk = self.packed(m)
        if self.bucket_lookup(m):
            return self.index.search_buckets(recv, m, cap, rcounts, algo="prefix" if pk else self.algo,
                                             out=buf["local"])
        if pk:  # without the bounded lookup every slot is searched
            return self.index.search_packed(recv, m, algo="prefix", out=buf["local"])
        return self.index.search_fixed(recv, m, algo=self.algo, out=buf["local"])

    def _backward(self, buf, local, async_op=False):
        if not self.exchange:
            return local, None
        w = self.dist.all_to_all_single(buf["back"], local, group=self.group, async_op=async_op)
        return buf["back"], w

    def search_fixed(self, qbytes, m: int, check: bool = True, out=None):
        """qbytes: uint8 tensor [nq*m] of this rank's queries -> int64 positions (written
        into `out` when given)."""
        if self.identity:
            return self._search_identity(qbytes, m, out)
        if not hasattr(self.index, "route_pack"):
            return self.search_fixed_exact(qbytes, m)
        if self.chunks > 1 and hasattr(self.index, "shard_gather"):
            return self._search_pipelined(qbytes, m, check, out)
        import torch
        nq = qbytes.numel() // m
        cap = self.capacity(nq)
        buf = self._buffers(m, cap)
        pk = self.packed(m)
        counts, send, slot = self.index.route_pack(self.splitters, qbytes, m, cap=cap, send=buf["send"],
                                                   **({"packed": True} if pk else {}))
        recv, rcounts, _ = self._forward(buf, send, counts)
        local = self._lookup(buf, recv, rcounts, m, cap)
        # what this rank received and answered in its last step (device tensors, no sync):
        # the bench proves a sample of them exact lower bounds on this part's own SA
        self.last = {"recv": recv, "rcounts": rcounts, "local": local, "cap": cap, "m": m, "packed": pk}
        back, _ = self._backward(buf, local)
        # one flag per step (check) or the sticky one (deferred to assert_no_overflow)
        flag = torch.zeros(1, dtype=torch.int32, device=self.device) if check else self.overflow
        if hasattr(self.index, "shard_gather"):  # gather + overflow test in one kernel
            out = self.index.shard_gather(back, slot, out=out, counts=counts, cap=cap, overflow=flag)
        else:
            flag |= (counts > cap).any().reshape(1).to(torch.int32)
            out = torch.index_select(back, 0, slot, out=out) if out is not None else back.index_select(0, slot)
        if check:
            # agreed by all (an overflow anywhere changes every rank's exchange): redo the
            # step with exact splits
            if self.world > 1:
                self.dist.all_reduce(flag, op=self.dist.ReduceOp.MAX, group=self.group)
            if int(flag.item()):
                exact = self.search_fixed_exact(qbytes, m)
                return out.copy_(exact) if out is not None else exact
        return out

    def _search_identity(self, qbytes, m: int, out):
        """World 1: every query is this rank's and lands in bucket 0 at its own index, so the
        lookup runs on the batch as given and its positions are the answer (no route, no
        gather; one piece whatever `chunks` says: there is no exchange to overlap)."""
        import torch
        nq = qbytes.numel() // m
        out = self.index.search_fixed(qbytes, m, algo=self.algo, out=out)
        key = ("identity", nq)
        if key not in self._bufs:
            self._bufs[key] = torch.full((1,), nq, dtype=torch.int64, device=self.device)
        # the one bucket this rank "received" (c4_proof samples it)
        self.last = {"recv": qbytes, "rcounts": self._bufs[key], "local": out, "cap": max(nq, 1), "m": m,
                     "packed": False}
        return out

    def _search_pipelined(self, qbytes, m: int, check: bool, out):
        """The step in `self.chunks` pieces of at most cs queries, one capacity for all:
        send sides and forward exchanges first (each exchange queued on the collective's
        stream as soon as its piece is packed), then per piece wait -> lookup -> backward
        exchange, then per piece wait -> gather into its slice of `out`."""
        import torch
        nq = qbytes.numel() // m
        C = self.chunks
        cs = -(-nq // C)
        cap = self.capacity(cs)
        pk = self.packed(m)
        if out is None:
            out = torch.empty(nq, dtype=torch.int64, device=self.device)
        flag = torch.zeros(1, dtype=torch.int32, device=self.device) if check else self.overflow
        pieces = []
        for c in range(C):
            s0, s1 = min(nq, c * cs), min(nq, (c + 1) * cs)
            buf = self._buffers(m, cap, c)
            counts, send, slot = self.index.route_pack(self.splitters, qbytes[s0 * m:s1 * m], m, cap=cap,
                                                       send=buf["send"], **({"packed": True} if pk else {}))
            recv, rcounts, works = self._forward(buf, send, counts, async_op=True)
            pieces.append((s0, s1, buf, counts, slot, recv, rcounts, works))
        back = []
        for s0, s1, buf, counts, slot, recv, rcounts, works in pieces:
            for w in works:
                w.wait()
            local = self._lookup(buf, recv, rcounts, m, cap)
            back.append(self._backward(buf, local, async_op=True))
        for (s0, s1, buf, counts, slot, *_), (bk, w) in zip(pieces, back):
            if w is not None:
                w.wait()
            if s1 > s0:
                self.index.shard_gather(bk, slot, out=out[s0:s1], counts=counts, cap=cap, overflow=flag)
        if check:
            if self.world > 1:
                self.dist.all_reduce(flag, op=self.dist.ReduceOp.MAX, group=self.group)
            if int(flag.item()):
                return out.copy_(self.search_fixed_exact(qbytes, m))
        return out

    def assert_no_overflow(self):
        """After steps run with check=False: every bucket fitted its capacity (so every
        result was exact)."""
        flag = self.overflow.clone()
        if self.world > 1:
            self.dist.all_reduce(flag, op=self.dist.ReduceOp.MAX, group=self.group)
        if int(flag.item()):
            raise RuntimeError("ShardedSearch: a bucket overflowed its capacity in a check=False step; "
                               "raise slack or run with check=True")
    def search_fixed_exact(self, qbytes, m: int):
        """Variable-size exchanges (counts first): exact for any routing, two host syncs."""
        import torch
        dist = self.dist
        if hasattr(self.index, "route_pack"):
            # GPU: routing, grouping by shard and the byte copy in one fused call
            send, qsend, slot = self.index.route_pack(self.splitters, qbytes, m)
        else:  # CPU stand-ins (tests): the same grouping with torch ops
            nq = qbytes.numel() // m
            dest = self.index.route(self.splitters, qbytes, m).to(torch.int64)
            order = torch.argsort(dest, stable=True)
            send = torch.bincount(dest, minlength=self.world)
            qsend = qbytes.view(nq, m).index_select(0, order).reshape(-1)
            slot = torch.empty_like(order)
            slot[order] = torch.arange(nq, device=order.device)
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self.group)
        send_l, recv_l = send.tolist(), recv.tolist()
        qrecv = torch.empty(sum(recv_l) * m, dtype=torch.uint8, device=qbytes.device)
        dist.all_to_all_single(qrecv, qsend, [c * m for c in recv_l], [c * m for c in send_l], group=self.group)
        local = self.index.search_fixed(qrecv, m, algo=self.algo) if sum(recv_l) else \
            torch.empty(0, dtype=torch.int64, device=qbytes.device)
        back = torch.empty(sum(send_l), dtype=torch.int64, device=qbytes.device)
        dist.all_to_all_single(back, local.to(torch.int64), send_l, recv_l, group=self.group)
        return back.index_select(0, slot)  # positions come back in send order
