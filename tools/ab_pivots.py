"""Same-box A/B of the pivot readers: PLAIN, LLCP and INLINE kernel times at n = 2^30, 10^7
positive queries (m = 32; LLCP also 64 / 128), at the library's default pivot depth and at
SAS_BUILD_TOP2_LEVELS(30) (keys name the depth the index reports), for the library under
AB_PKG (a tools/mk_variant.sh build, or a git-archive build of another commit) or the tree's:
    AB_PKG=tools/_var_<name>/suffix-array-searching_amd python3 tools/ab_pivots.py"""
import json
import os
import sys

sys.path.insert(0, os.environ.get("AB_PKG") or
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "suffix-array-searching_amd"))
import numpy as np
import torch

import sas_amd

n, nq = 1 << 30, 10_000_000
t = sas_amd.random_string(n, seed=31415, device="cuda")
res = {"pkg": os.environ.get("AB_PKG", "tree"), "source_hash": sas_amd.source_hash()}
qs = {}
for m in (32, 64, 128):
    off, _, _ = sas_amd.random_queries(n, nq, seed=31415, word_pos=n, margin=256, len_lo=m, len_hi=m + 1)
    src = torch.from_numpy(off.astype(np.int64)).cuda()
    qs[m] = t[(src[:, None] + torch.arange(m, device="cuda")[None, :]).reshape(-1)].contiguous()
out = torch.empty(nq, dtype=torch.int64, device="cuda")
for L in (0, 30):
    idx = sas_amd.SaNaive.build(t, lcp=True, stree=False, sector=False, quad=True, llcp=True, prefix=False,
                                top2_levels=L)
    ref = None
    for algo, m in (("plain", 32), ("llcp", 32), ("inline", 32), ("llcp", 64), ("llcp", 128), ("plain", 128)):
        idx.time_fixed(qs[m], m, nq, out, algo=algo, reps=3)
        kns, _ = idx.time_fixed(qs[m], m, nq, out, algo=algo, reps=20)
        res[f"L{idx.stats()['top2_levels']}_{algo}_m{m}"] = round(kns / 1e6, 4)
        if m == 32:
            if ref is None:
                ref = out.clone()
            assert torch.equal(out, ref), (L, algo)
    idx.free()
    torch.cuda.empty_cache()
print(json.dumps(res), flush=True)
