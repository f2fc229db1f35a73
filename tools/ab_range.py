"""Occurrence-range throughput (sas_search_range, Search::search_prefix) at the c1 shape:
prefix-table bounds vs the quad-tree descents (SAS_NO_PREFIX_TABLE), same index."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "suffix-array-searching_amd"))
import numpy as np
import torch

import sas_amd
from sas_amd import _lib

n, nq, m = 1 << 30, 10_000_000, 32
t = sas_amd.random_string(n, seed=31415, device="cuda")
off, _, _ = sas_amd.random_queries(n, nq, seed=31415, word_pos=n, margin=200, len_lo=m, len_hi=m + 1)
src = torch.from_numpy(off.astype(np.int64)).cuda()
qb = t[(src[:, None] + torch.arange(m, device="cuda")[None, :]).reshape(-1)].contiguous()
qoff = torch.arange(nq, device="cuda", dtype=torch.int64) * m
qlen = torch.full((nq,), m, dtype=torch.int32, device="cuda")
idx = sas_amd.SaNaive.build(t, lcp=False, stree=False, sector=False, llcp=False, quad=True, prefix=16, prefix_inline=2)
res = {}
for name, fl in (("prefix_table", 0), ("quad_descents", _lib.SAS_NO_PREFIX_TABLE), ("prefix_table2", 0)):
    idx.search_range(qb, qoff, qlen, flags=fl)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        lo, hi = idx.search_range(qb, qoff, qlen, flags=fl)
    e1.record()
    torch.cuda.synchronize()
    res[name] = round(e0.elapsed_time(e1) / 5, 4)
    res[name + "_sum"] = int((hi - lo).sum().item())
print("ms", res, flush=True)
