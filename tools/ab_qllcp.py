"""Same-box A/B of configs[2]'s long-query kernels -- QUAD (k_sa_quad4x), STREE_LLCP
(k_sa_stree4x<.., true>) and QUAD_LLCP (k_sa_quad_llcp) -- at n = 2^30, 10^7 positive queries
of m = 64 / 128 / 256 chars, on the bench's random text and its repetitive text (2^24 random
chars x 64 copies, 1% substitutions: benchlib.records.repetitive_text), for the libraries under
AB_PKGS (colon-separated tools/mk_variant.sh builds; 'tree' = this tree's), interleaved round
robin over AB_ROUNDS rounds.  Positions must equal QUAD's.  One JSON line per text:
{"text": ..., "<pkg>": {"<algo>_m<m>": [ms per round]}}.
    AB_PKGS=tree:tools/_var_l512/suffix-array-searching_amd python3 tools/ab_qllcp.py"""
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
pkgs = os.environ.get("AB_PKGS", "tree").split(":")
algos = os.environ.get("AB_ALGOS", "quad,stree_llcp,quad_llcp").split(",")
ms = [int(x) for x in os.environ.get("AB_MS", "64,128,256").split(",")]
texts = os.environ.get("AB_TEXTS", "random,repetitive").split(",")
rounds = int(os.environ.get("AB_ROUNDS", "3"))
reps = int(os.environ.get("AB_REPS", "10"))
n, nq = 1 << 30, 10_000_000


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
for tname in texts:
    if tname == "random":
        t = base.random_string(n, seed=31415, device="cuda")
    else:
        from benchlib.records import repetitive_text
        t = repetitive_text(torch, n, torch.device("cuda"))
    qs = {}
    for m in ms:
        off, _, _ = base.random_queries(n, nq, seed=31415, word_pos=n, margin=256, len_lo=m, len_hi=m + 1)
        src = torch.from_numpy(off.astype(np.int64)).cuda()
        q = torch.empty(nq * m, dtype=torch.uint8, device="cuda")
        ar = torch.arange(m, device="cuda")
        step = (1 << 23) // m
        for s0 in range(0, nq, step):
            e0 = min(nq, s0 + step)
            q[s0 * m:e0 * m] = t[(src[s0:e0, None] + ar[None, :]).reshape(-1)]
        qs[m] = q
    need_stree = any(a.startswith("stree") for a in algos)
    out = torch.empty(nq, dtype=torch.int64, device="cuda")
    res = {"text": tname}
    ref = {}
    for p in pkgs:
        res[p] = {"source_hash": mods[p].source_hash()}
    idx = {}
    for p in pkgs:
        idx[p] = mods[p].SaNaive.build(t, lcp=True, stree=need_stree, sector=False, quad=True, llcp=True, prefix=False)
    for rd in range(rounds):
        for p in pkgs:
            ix = idx[p]
            for m in ms:
                for algo in algos:
                    ix.time_fixed(qs[m], m, nq, out, algo=algo, reps=2)
                    kns, _ = ix.time_fixed(qs[m], m, nq, out, algo=algo, reps=reps)
                    res[p].setdefault(f"{algo}_m{m}", []).append(round(kns / 1e6, 4))
                    ix.time_fixed(qs[m], m, nq, out, algo=algo, reps=1)
                    if m not in ref:
                        ref[m] = out.clone()
                    assert torch.equal(out, ref[m]), (tname, p, algo, m)
    print(json.dumps(res), flush=True)
    for p in pkgs:
        idx[p].free()
    del t, qs, idx
    torch.cuda.empty_cache()
