"""A/B: kernel time of one algorithm with and without other trees built beside it
(tests whether co-resident index memory slows the random-access kernels)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "suffix-array-searching_amd"))
import numpy as np
import torch
import sas_amd

n, nq, m = 1 << 30, 10_000_000, 32
t = sas_amd.random_string(n, seed=31415, device="cuda")
off, _, _ = sas_amd.random_queries(n, nq, seed=31415, word_pos=n, margin=200, len_lo=m, len_hi=m + 1)
src = torch.from_numpy(off.astype(np.int64)).cuda()
qb = t[(src[:, None] + torch.arange(m, device="cuda")[None, :]).reshape(-1)].contiguous()
out = torch.empty(nq, dtype=torch.int64, device="cuda")
for cfg in [dict(sector=True, quad=False, stree=False, lcp=False), dict(sector=False, quad=True, stree=False, lcp=False),
            dict(sector=True, quad=True, stree=True, lcp=True)]:
    idx = sas_amd.SaNaive.build(t, **cfg)
    for algo in ("sector", "quad"):
        if not cfg[algo]:
            continue
        idx.time_fixed(qb, m, nq, out, algo=algo, reps=3)
        kns, _ = idx.time_fixed(qb, m, nq, out, algo=algo, reps=20)
        print(cfg, algo, f"{kns / 1e6:.4f} ms", flush=True)
    idx.free()
    torch.cuda.empty_cache()
