"""PREFIX and QUAD kernel times at the configs[3] shape (n = 2^34 chars, 40-bit SA,
compact quad leaves, p = 16 prefix table, ragged 8..256 queries) for same-box A/B of
library builds: AB_PKG=tools/_var_<name>/suffix-array-searching_amd AB_NQ=20000000
python3 tools/ab_c3.py"""
import os
import sys

sys.path.insert(0, os.environ.get("AB_PKG") or
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "suffix-array-searching_amd"))
import numpy as np
import torch

import sas_amd

n = int(os.environ.get("AB_N", 1 << 34))
nq = int(os.environ.get("AB_NQ", 20_000_000))
t = sas_amd.random_string(n, seed=31415, device="cuda")
idx = sas_amd.SaNaive.build(t, lcp=False, stree=False, sector=False, quad="compact", llcp=False, prefix=16)
del t
torch.cuda.empty_cache()
off, ln, _ = sas_amd.random_queries(n, nq, seed=31415, word_pos=n, margin=256, len_lo=8, len_hi=257)
lens = torch.from_numpy(ln.astype(np.int32)).cuda()
qoff = torch.zeros(nq, dtype=torch.int64, device="cuda")
qoff[1:] = torch.cumsum(lens.long(), 0)[:-1]
qb = torch.zeros(int(lens.sum().item()) + 64, dtype=torch.uint8, device="cuda")
idx.extract(torch.from_numpy(off.astype(np.int64)).cuda(), lens, qoff, qb)
out = torch.empty(nq, dtype=torch.int64, device="cuda")
line = {}
ref = None
for algo in ("prefix", "quad", "prefix", "quad"):
    idx.search_batch(qb, qoff, lens, algo=algo, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        idx.search_batch(qb, qoff, lens, algo=algo, out=out)
    e1.record()
    torch.cuda.synchronize()
    line.setdefault(algo, []).append(round(e0.elapsed_time(e1) / 3, 3))
    ref = out.clone() if ref is None else ref
    line[algo + "_ok"] = bool(torch.equal(out, ref))
print("ms", line, flush=True)
