"""Kernel times of PREFIX (and QUAD beside it) at the c1 shape (2^30 text, 10^7 len-32
queries) for same-box A/B of library builds:
AB_PKG=tools/_var_<name>/suffix-array-searching_amd python3 tools/ab_prefix.py"""
import os
import sys

sys.path.insert(0, os.environ.get("AB_PKG") or
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "suffix-array-searching_amd"))
import numpy as np
import torch

import sas_amd

n, nq, m = 1 << 30, 10_000_000, 32
# PROBE_BALLAST_GB: device memory held before the text and index (placement probe)
_bg = float(os.environ.get("PROBE_BALLAST_GB", "0"))
ballast = torch.empty(int(_bg * 2**30), dtype=torch.uint8, device="cuda") if _bg else None
t = sas_amd.random_string(n, seed=31415, device="cuda")
off, _, _ = sas_amd.random_queries(n, nq, seed=31415, word_pos=n, margin=200, len_lo=m, len_hi=m + 1)
src = torch.from_numpy(off.astype(np.int64)).cuda()
qb = t[(src[:, None] + torch.arange(m, device="cuda")[None, :]).reshape(-1)].contiguous()
out = torch.empty(nq, dtype=torch.int64, device="cuda")
# AB_MODES: comma list of <p><r|i|d|q>: ranks-only (u32), or inline entries holding the
# first 1 / 2 / 4 suffixes of each range (16 / 32 / 64 B)
for mode in os.environ.get("AB_MODES", "16r").split(","):
    p, inl = int(mode[:-1]), {"r": 0, "i": 1, "d": 2, "q": 4}[mode[-1]]
    idx = sas_amd.SaNaive.build(t, lcp=False, stree=False, sector=False, llcp=False, quad=True, prefix=p,
                                prefix_inline=inl)
    line = {"mode": mode, "p": idx.stats()["prefix_chars"], "ballast_gb": _bg}
    ref = None
    for algo in ("prefix", "quad"):
        idx.time_fixed(qb, m, nq, out, algo=algo, reps=2)
        kns, _ = idx.time_fixed(qb, m, nq, out, algo=algo, reps=10)
        line[algo] = round(kns / 1e6, 4)
        ref = out.clone() if ref is None else ref
        line[algo + "_ok"] = bool(torch.equal(out, ref))
    print("ms", line, flush=True)
    idx.free()
    torch.cuda.empty_cache()
