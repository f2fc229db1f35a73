"""Same-box A/B of the binary-search kernels (k_sa_binary: PLAIN, LCP, LLCP; and INLINE) at
n = 2^30, 10^7 positive queries, the library's default pivot depth, for the libraries under
AB_PKGS (colon-separated tools/mk_variant.sh builds; 'tree' = this tree's), interleaved
round-robin over AB_ROUNDS rounds so box drift hits every library alike.  Positions must equal
PLAIN's on the same queries.  One JSON line: {"<pkg>": {"<algo>_m<m>": [ms per round]}}.
    AB_PKGS=tree:tools/_var_b768/suffix-array-searching_amd python3 tools/ab_bin.py"""
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
pkgs = os.environ.get("AB_PKGS", "tree").split(":")
cases = [c.split("@") for c in os.environ.get(
    "AB_CASES", "plain@32,llcp@32,lcp@32,inline@32,plain@64,llcp@64,llcp@128,plain@128").split(",")]
rounds = int(os.environ.get("AB_ROUNDS", "3"))
reps = int(os.environ.get("AB_REPS", "20"))


def load(p):
    path = os.path.join(ROOT, "suffix-array-searching_amd") if p == "tree" else os.path.join(ROOT, p)
    for k in [k for k in sys.modules if k == "sas_amd" or k.startswith("sas_amd.")]:
        del sys.modules[k]
    sys.path.insert(0, path)
    mod = importlib.import_module("sas_amd")
    sys.path.pop(0)
    return mod


mods = {p: load(p) for p in pkgs}
base = mods[pkgs[0]]
n, nq = 1 << 30, 10_000_000
t = base.random_string(n, seed=31415, device="cuda")
qs = {}
for m in sorted({int(m) for _, m in cases}):
    off, _, _ = base.random_queries(n, nq, seed=31415, word_pos=n, margin=256, len_lo=m, len_hi=m + 1)
    src = torch.from_numpy(off.astype(np.int64)).cuda()
    qs[m] = t[(src[:, None] + torch.arange(m, device="cuda")[None, :]).reshape(-1)].contiguous()
need_llcp = any(a == "llcp" for a, _ in cases)
need_llcp = need_llcp or any(a == "stree_llcp" for a, _ in cases)
need_quad = any(a in ("inline", "quad") for a, _ in cases)
need_stree = any(a.startswith("stree") for a, _ in cases)
idx = {p: mods[p].SaNaive.build(t, lcp=True, stree=need_stree, sector=False, quad=need_quad, llcp=need_llcp,
                                 prefix=False) for p in pkgs}
out = torch.empty(nq, dtype=torch.int64, device="cuda")
res = {p: {"source_hash": mods[p].source_hash()} for p in pkgs}
ref = {}
for rd in range(rounds):
    for p in pkgs:
        for algo, m in cases:
            m = int(m)
            ix = idx[p]
            ix.time_fixed(qs[m], m, nq, out, algo=algo, reps=2)
            kns, _ = ix.time_fixed(qs[m], m, nq, out, algo=algo, reps=reps)
            res[p].setdefault(f"{algo}_m{m}", []).append(round(kns / 1e6, 4))
            if m not in ref:
                ix.time_fixed(qs[m], m, nq, out, algo="plain", reps=1)
                ref[m] = out.clone()
                ix.time_fixed(qs[m], m, nq, out, algo=algo, reps=1)
            assert torch.equal(out, ref[m]), (p, algo, m)
print(json.dumps(res), flush=True)
