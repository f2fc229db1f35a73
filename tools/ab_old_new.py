"""Same-box A/B of the sector kernel: this tree's library vs an older build
(tools/_old, from `git archive`), same text, queries and timing helper."""
import sys, os
which = sys.argv[1]
algo = sys.argv[2] if len(sys.argv) > 2 else "sector"
shape = sys.argv[3] if len(sys.argv) > 3 else "c1"   # c1: len-32 fixed; c3: ragged 8..256
qmode = sys.argv[4] if len(sys.argv) > 4 else "fused"  # quad leaves: fused | compact
root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_" + which if which.startswith("old") else "..")
sys.path.insert(0, os.path.join(root, "suffix-array-searching_amd"))
import numpy as np
import torch
import sas_amd
print(which, sas_amd.__file__)
ref = None
n, nq, m = 1 << 30, 10_000_000, 32
t = sas_amd.random_string(n, seed=31415, device="cuda")
if shape == "c1":
    off, _, _ = sas_amd.random_queries(n, nq, seed=31415, word_pos=n, margin=200, len_lo=m, len_hi=m + 1)
    src = torch.from_numpy(off.astype(np.int64)).cuda()
    qb = t[(src[:, None] + torch.arange(m, device="cuda")[None, :]).reshape(-1)].contiguous()
else:
    off, ln, _ = sas_amd.random_queries(n, nq, seed=31415, word_pos=n, margin=300, len_lo=8, len_hi=257)
    lens = torch.from_numpy(ln.astype(np.int64)).cuda()
    qoff = torch.zeros(nq, dtype=torch.int64, device="cuda")
    qoff[1:] = torch.cumsum(lens, 0)[:-1]
    src = torch.from_numpy(off.astype(np.int64)).cuda()
    rep = torch.repeat_interleave(torch.arange(nq, device="cuda"), lens)
    within = torch.arange(rep.numel(), device="cuda") - qoff[rep]
    qb = torch.cat([t[src[rep] + within], torch.zeros(64, dtype=torch.uint8, device="cuda")])
    qlen = lens.to(torch.int32)
out = torch.empty(nq, dtype=torch.int64, device="cuda")
kw = dict(sector=algo == "sector", stree=algo == "stree", lcp=False, quad=("compact" if qmode == "compact" else True) if algo in ("quad", "inline") else False)
idx = sas_amd.SaNaive.build(t, **kw)
import time
for r in range(3):
    if shape == "c1":
        idx.time_fixed(qb, m, nq, out, algo=algo, reps=3)
        kns, _ = idx.time_fixed(qb, m, nq, out, algo=algo, reps=20)
    else:
        idx.search_batch(qb, qoff, qlen, algo=algo, out=out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            idx.search_batch(qb, qoff, qlen, algo=algo, out=out)
        e1.record()
        torch.cuda.synchronize()
        kns = e0.elapsed_time(e1) / 5 * 1e6
    print(which, algo, shape, qmode, f"{kns / 1e6:.4f} ms", flush=True)
np.save(f"/tmp/ab_{which}_{algo}_{shape}_{qmode}.npy", out.cpu().numpy())
