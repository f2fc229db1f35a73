"""Sharded-text mode: the suffix array is split into SA-rank ranges,
one per GPU; queries are routed to the GPU owning their lower bound and the
positions come back -- the only place this engine uses a collective.

    rank g holds global SA ranks [g*n/W, (g+1)*n/W) (SaNaive.build(rank_range=...)),
    splitters = text positions of the first suffix of shards 1..W-1 (all-gathered once),
    step: route (sas_route) -> group by destination -> all_to_all counts, query bytes
          -> local lookup -> all_to_all positions back -> restore query order.

Hash-partitioning the SA would break its order (a lower bound would need every
shard); rank ranges keep each answer on exactly one shard.  The collective is
`torch.distributed.all_to_all_single` (RCCL over xGMI with backend "nccl";
gloo in the CPU tests).  Payload per query: m bytes out, 8 bytes back.
"""
from __future__ import annotations


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Global SA ranks owned by `rank`: contiguous and balanced."""
    return (n * rank) // world, (n * (rank + 1)) // world


class ShardedSearch:
    """`index` needs: .route(splitters, qbytes, m) -> dest shard per query,
    .search_fixed(qbytes, m, algo=...) -> positions (int64), .suffix_array(1) ->
    its first SA value.  The GPU implementation is sas_amd.SaNaive."""

    def __init__(self, index, dist, world: int, rank: int, device, algo: str = "stree", group=None):
        import torch
        self.index, self.dist, self.world, self.rank = index, dist, world, rank
        self.device, self.algo, self.group = device, algo, group
        first = torch.tensor([int(index.suffix_array(1)[0])], dtype=torch.int64, device=device)
        firsts = [torch.empty_like(first) for _ in range(world)]
        dist.all_gather(firsts, first, group=group)
        # first suffix of shards 1..W-1, in increasing suffix order
        self.splitters = torch.cat(firsts[1:]).to(torch.int64) if world > 1 else torch.empty(0, dtype=torch.int64,
                                                                                              device=device)

    def search_fixed(self, qbytes, m: int):
        """qbytes: uint8 tensor [nq*m] of this rank's queries -> int64 positions."""
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
