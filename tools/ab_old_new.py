"""Same-box A/B of the sector kernel: this tree's library vs an older build
(tools/_old, from `git archive`), same text, queries and timing helper."""
import sys, os
which = sys.argv[1]
algo = sys.argv[2] if len(sys.argv) > 2 else "sector"
root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_old" if which == "old" else "..")
sys.path.insert(0, os.path.join(root, "suffix-array-searching_amd"))
import numpy as np
import torch
import sas_amd
print(which, sas_amd.__file__)
ref = None
n, nq, m = 1 << 30, 10_000_000, 32
t = sas_amd.random_string(n, seed=31415, device="cuda")
off, _, _ = sas_amd.random_queries(n, nq, seed=31415, word_pos=n, margin=200, len_lo=m, len_hi=m + 1)
src = torch.from_numpy(off.astype(np.int64)).cuda()
qb = t[(src[:, None] + torch.arange(m, device="cuda")[None, :]).reshape(-1)].contiguous()
out = torch.empty(nq, dtype=torch.int64, device="cuda")
kw = dict(sector=algo == "sector", stree=algo == "stree", lcp=False, quad=algo == "quad")
idx = sas_amd.SaNaive.build(t, **kw)
for rep in range(3):
    idx.time_fixed(qb, m, nq, out, algo=algo, reps=3)
    kns, _ = idx.time_fixed(qb, m, nq, out, algo=algo, reps=20)
    print(which, algo, f"{kns / 1e6:.4f} ms", flush=True)
np.save(f"/tmp/ab_{which}_{algo}.npy", out.cpu().numpy())
