"""Where configs[4]'s N = 1 step spends its time: the step as the bench times it (event pair
around K steps; round 6: the world-1 identity step, the part's lookup alone), the routed shape
each rank of a W > 1 step runs (routed=True: route + identity exchange + gather), the host's
enqueue time for K steps (no sync inside), each piece alone (route, lookup, gather), the route
and gather at the W = 8 shape on this one part (7 splitters = the SA values at ranks j n / 8,
8 buckets of 1.125 nq / 8 + 256 slots: what an 8-GPU rank's send and receive sides cost), and
the routed step replayed from a HIP graph (torch.cuda.CUDAGraph).  One JSON line.
usage: c4_step_probe.py [share_log2=30]   (GPU box)"""
import json
import os
import socket
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "suffix-array-searching_amd"))
import bench  # noqa: E402
import sas_amd  # noqa: E402
import torch.distributed as dist  # noqa: E402
from sas_amd.shard import ShardedSearch  # noqa: E402

share = 1 << (int(sys.argv[1]) if len(sys.argv) > 1 else 30)
n, nq, m, K = share, 10_000_000, 32, 20
dev = torch.device("cuda:0")
sk = socket.socket()
sk.bind(("127.0.0.1", 0))
port = sk.getsockname()[1]
sk.close()
dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
idx = sas_amd.SaNaive.build_part_gen(n, seed=bench.SEED + 1, part=0, parts=1, lcp=False, stree=False, sector=False,
                                     quad=True, llcp=False, prefix=16, prefix_inline=2,
                                     top2_levels=bench.TOP_LDS_LEVELS)
off = torch.from_numpy(bench.rank_query_offsets(n, nq, m, 0).astype(np.int64)).to(dev)
q = torch.empty(nq * m, dtype=torch.uint8, device=dev)
idx.extract(off, torch.full((nq,), m, dtype=torch.int32, device=dev),
            torch.arange(nq, device=dev, dtype=torch.int64) * m, q)
eng = ShardedSearch(idx, dist, 1, 0, dev, algo="prefix", chunks=1, max_nq=nq)
assert eng.identity
engr = ShardedSearch(idx, dist, 1, 0, dev, algo="prefix", chunks=1, max_nq=nq, routed=True)
out = torch.empty(nq, dtype=torch.int64, device=dev)
res = {"n": n, "nq": nq, "source_hash": sas_amd.source_hash()}


def ev_time(fn, k=K):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    h0 = time.perf_counter()
    a.record()
    for _ in range(k):
        fn()
    h1 = time.perf_counter()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / k, (h1 - h0) * 1e3 / k


res["step_ms"], res["step_host_enqueue_ms"] = ev_time(lambda: eng.search_fixed(q, m, check=False, out=out))
ref = out.clone()
# the replicated headline's kernel on the same batch (the identity step's target)
res["replicated_lookup_ms"], _ = ev_time(lambda: idx.search_fixed(q, m, algo="prefix", out=out))
assert torch.equal(out, ref)
step = lambda: engr.search_fixed(q, m, check=False, out=out)  # noqa: E731
res["routed_step_ms"], res["routed_step_host_enqueue_ms"] = ev_time(step)
assert torch.equal(out, ref)
eng = engr
cap = eng.capacity(nq)
buf = eng._buffers(m, cap)
counts, send, slot = idx.route_pack(eng.splitters, q, m, cap=cap, send=buf["send"], packed=True)
res["route_ms"], res["route_host_ms"] = ev_time(
    lambda: idx.route_pack(eng.splitters, q, m, cap=cap, send=buf["send"], packed=True))
res["lookup_ms"], res["lookup_host_ms"] = ev_time(lambda: eng._lookup(buf, send, counts, m, cap))
local = eng._lookup(buf, send, counts, m, cap)
res["gather_ms"], res["gather_host_ms"] = ev_time(
    lambda: idx.shard_gather(local, slot, out=out, counts=counts, cap=cap, overflow=eng.overflow))
# the W = 8 shape on this part: 7 splitters, 8 fixed-capacity buckets (packed words)
W8 = 8
sa_n = idx.stats()["sa_entries"]
sp8 = torch.tensor([int(idx.suffix_array(count=1, start=(j * sa_n) // W8)[0]) for j in range(1, W8)],
                   dtype=torch.int64, device=dev)
cap8 = int(nq * ShardedSearch.SLACK / W8) + 256
send8 = torch.zeros(W8 * cap8, dtype=torch.int64, device=dev)
res["w8_route_ms"], res["w8_route_host_ms"] = ev_time(
    lambda: idx.route_pack(sp8, q, m, cap=cap8, send=send8, packed=True))
c8, s8, slot8 = idx.route_pack(sp8, q, m, cap=cap8, send=send8, packed=True)
res["w8_counts"] = c8.cpu().tolist()
back8 = torch.zeros(W8 * cap8, dtype=torch.int64, device=dev)
flag8 = torch.zeros(1, dtype=torch.int32, device=dev)
res["w8_gather_ms"], _ = ev_time(lambda: idx.shard_gather(back8, slot8, out=out, counts=c8, cap=cap8, overflow=flag8))
res["w8_overflow"] = int(flag8.item())
# the routed step captured once and replayed
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        step()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
try:
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    out.zero_()
    res["graph_ms"], res["graph_host_ms"] = ev_time(g.replay)
    res["graph_identical"] = bool(torch.equal(out, ref))
except Exception as e:  # noqa: BLE001
    res["graph_error"] = repr(e)[:300]
eng.assert_no_overflow()
print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
dist.destroy_process_group()
