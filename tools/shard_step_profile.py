"""Time the pieces of one sharded-mode step (ws = 1: RCCL all_to_all is a local copy)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "suffix-array-searching_amd"))
import numpy as np
import torch
import torch.distributed as dist
import sas_amd
from sas_amd.shard import ShardedSearch

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29531")
dist.init_process_group("nccl", rank=0, world_size=1)
dev = torch.device("cuda", 0)
n, nq, m = 1 << 30, 10_000_000, 32
t = sas_amd.random_string(n, seed=31415, device=dev)
idx = sas_amd.SaNaive.build_part(t, 0, 1, lcp=False, stree=False, sector=False, quad=True)
off, _, _ = sas_amd.random_queries(n, nq, seed=31415, word_pos=n, margin=200, len_lo=m, len_hi=m + 1)
src = torch.from_numpy(off.astype(np.int64)).to(dev)
qb = t[(src[:, None] + torch.arange(m, device=dev)[None, :]).reshape(-1)].contiguous()
eng = ShardedSearch(idx, dist, 1, 0, dev, algo="quad")
for _ in range(3):
    eng.search_fixed(qb, m)
torch.cuda.synchronize()


def tm(label, fn, reps=5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = fn()
    torch.cuda.synchronize()
    print(f"{label:28s} {(time.perf_counter() - t0) / reps * 1e3:8.3f} ms", flush=True)
    return r


dest = tm("route", lambda: idx.route(eng.splitters, qb, m).to(torch.int64))
tm("argsort int64 stable", lambda: torch.argsort(dest, stable=True))
tm("sort uint8 stable", lambda: torch.sort(dest.to(torch.uint8), stable=True))
tm("bincount", lambda: torch.bincount(dest, minlength=1))
order = torch.argsort(dest, stable=True)
tm("index_select queries", lambda: qb.view(nq, m).index_select(0, order).reshape(-1))
tm("search quad", lambda: idx.search_fixed(qb, m, algo="quad"))
tm("full step", lambda: eng.search_fixed(qb, m))
dist.destroy_process_group()
