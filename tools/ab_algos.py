"""Kernel times of every SA algorithm (c1: 2^30 text, 10^7 len-32 queries) and of the
u32 STree16 left_max / PartitionedSTree16M (2^28 keys, 10^7 queries), for same-box A/B
of library builds: AB_PKG=tools/_var_<name>/suffix-array-searching_amd python3 tools/ab_algos.py"""
import os
import sys

sys.path.insert(0, os.environ.get("AB_PKG") or
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "suffix-array-searching_amd"))
import numpy as np
import torch

import sas_amd

n, nq, m = 1 << 30, 10_000_000, 32
t = sas_amd.random_string(n, seed=31415, device="cuda")
off, _, _ = sas_amd.random_queries(n, nq, seed=31415, word_pos=n, margin=200, len_lo=m, len_hi=m + 1)
src = torch.from_numpy(off.astype(np.int64)).cuda()
qb = t[(src[:, None] + torch.arange(m, device="cuda")[None, :]).reshape(-1)].contiguous()
out = torch.empty(nq, dtype=torch.int64, device="cuda")
idx = sas_amd.SaNaive.build(t, lcp=True, stree=True, sector=True, quad=True)
line = {}
for algo in ("quad", "sector", "stree", "inline", "plain"):
    idx.time_fixed(qb, m, nq, out, algo=algo, reps=2)
    kns, _ = idx.time_fixed(qb, m, nq, out, algo=algo, reps=10)
    line[algo] = round(kns / 1e6, 4)
idx.free()
del t, qb, out
torch.cuda.empty_cache()
rng = np.random.default_rng(31415)
vals = np.sort(rng.integers(0, 2**31 - 1, 1 << 28, dtype=np.uint64).astype(np.uint32))
vals[-1] = 2**31 - 1
qs = torch.from_numpy(rng.integers(0, 2**31 - 1, nq, dtype=np.uint64).astype(np.uint32).view(np.int32)).cuda()
dout = torch.empty(nq, dtype=torch.int32, device="cuda")
for name, mk in (("stree16lm", lambda: sas_amd.STree16.new_params(vals, True, False, False)),
                 ("pmap16", lambda: sas_amd.PartitionedSTree16M.new(vals, 16))):
    ix = mk()
    ix.time_query(qs, dout, reps=2)
    line[name] = round(ix.time_query(qs, dout, reps=10) * 1e-6, 4)
    ix.free()
print("ms", line, flush=True)
