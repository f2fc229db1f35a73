"""PLAIN vs LCP (Manber-Myers mlr skipping) on a random text and a repeat-rich one
(a 2^20-char block tiled with 1% point mutations), positive queries of length m."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "suffix-array-searching_amd"))
import numpy as np
import torch

import sas_amd

n, nq = 1 << 28, 2_000_000
rng = np.random.default_rng(5)
blk = rng.integers(0, 4, 1 << 20, dtype=np.uint8)
rep = np.tile(blk, n >> 20)
mut = rng.integers(0, n, n // 100)
rep[mut] = rng.integers(0, 4, len(mut), dtype=np.uint8)
for name, t in (("random", sas_amd.random_string(n, seed=9, device="cuda")), ("repeats", torch.from_numpy(rep).cuda())):
    idx = sas_amd.SaNaive.build(t, lcp=True, stree=False, sector=False, quad=False)
    for m in (32, 128, 256):
        off = torch.from_numpy(rng.integers(0, n - m - 1, nq)).cuda()
        qb = t[(off[:, None] + torch.arange(m, device="cuda")[None, :]).reshape(-1)].contiguous()
        out = torch.empty(nq, dtype=torch.int64, device="cuda")
        res = {}
        for algo in ("plain", "lcp"):
            idx.time_fixed(qb, m, nq, out, algo=algo, reps=1)
            kns, _ = idx.time_fixed(qb, m, nq, out, algo=algo, reps=5)
            res[algo] = round(kns / 1e6, 3)
        print(name, "m", m, "ms", res, flush=True)
    idx.free()
    torch.cuda.empty_cache()
