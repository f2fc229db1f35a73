"""Rehearse one rank of the driver's 8-GPU configs[4] record on one GPU: the 2^33-char
text (8 x the per-GPU share), this rank's part (sas_build_part, the bench's flags), setup
time, index bytes, and the local PREFIX lookup of 10^7 packed len-32 queries (the part's
share of a step).  usage: c4_part_probe.py [parts] [part] [inline]   (GPU box)"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "suffix-array-searching_amd")
import sas_amd  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
g = int(sys.argv[2]) if len(sys.argv) > 2 else W - 1
n, nq, m = (1 << 30) * W, 10_000_000, 32
t0 = time.perf_counter()
text = sas_amd.random_string(n, seed=31416, device="cuda")
torch.cuda.synchronize()
t1 = time.perf_counter()
inline = int(sys.argv[3]) if len(sys.argv) > 3 else 2  # 0: the 40-bit rank table
idx = sas_amd.SaNaive.build_part(text, g, W, lcp=False, stree=False, sector=False, quad=True, llcp=False, prefix=16,
                                 prefix_inline=inline)
torch.cuda.synchronize()
t2 = time.perf_counter()
st = idx.stats()
rng = np.random.default_rng(2)
off = torch.from_numpy(rng.integers(0, n - m, nq)).cuda()
ar = torch.arange(m, device="cuda")
q = torch.empty(nq * m, dtype=torch.uint8, device="cuda")
for s in range(0, nq, 1 << 18):
    e = min(nq, s + (1 << 18))
    q[s * m:e * m] = text[(off[s:e, None] + ar[None, :]).reshape(-1)]
w = sas_amd.SaNaive.pack_queries(q, m)
out = torch.empty(nq, dtype=torch.int64, device="cuda")
for _ in range(3):
    idx.search_packed(w, m, out=out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    idx.search_packed(w, m, out=out)
e1.record()
torch.cuda.synchronize()
print(json.dumps({"parts": W, "part": g, "n": n, "text_s": round(t1 - t0, 2), "build_part_s": round(t2 - t1, 2),
                  "sa_entries": st["sa_entries"], "sa_width": st["sa_width"], "prefix_chars": st["prefix_chars"],
                  "prefix_bytes": st["prefix_bytes"], "index_bytes": st["index_bytes"],
                  "local_prefix_packed_ms": round(e0.elapsed_time(e1) / 10, 4),
                  "max_allocated_GiB": round(torch.cuda.max_memory_allocated() / 2**30, 1)}), flush=True)
