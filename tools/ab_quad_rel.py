"""Same-box A/B: quad tree with prefix-relative 31-ary inner nodes (SAS_BUILD_QUAD_REL) vs
the 17-ary absolute layout (SAS_BUILD_QUAD_ABS), fused and compact leaves, on the c1
workload (2^30 text, 10^7 len-32 queries) and a ragged 8..256 sample.  Alternates
the two indexes so box drift hits both; checks the positions are identical."""
import os
import sys

# AB_PKG: another build of the package (tools/mk_variant.sh) to time instead of this tree's
sys.path.insert(0, os.environ.get("AB_PKG") or
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "suffix-array-searching_amd"))
import numpy as np
import torch

import sas_amd

n, nq, m = int(os.environ.get("AB_N", 1 << 30)), 10_000_000, 32
leaves = os.environ.get("AB_LEAVES", "fused")
t = sas_amd.random_string(n, seed=31415, device="cuda")
off, _, _ = sas_amd.random_queries(n, nq, seed=31415, word_pos=n, margin=200, len_lo=m, len_hi=m + 1)
src = torch.from_numpy(off.astype(np.int64)).cuda()
qb = t[(src[:, None] + torch.arange(m, device="cuda")[None, :]).reshape(-1)].contiguous()
out = torch.empty(nq, dtype=torch.int64, device="cuda")
pre = "" if leaves == "fused" else "compact-"
kinds = {"rel": pre + "rel", "abs": pre + "abs"}
# AB_SEQ=1: one index at a time (n = 2^34: two compact quad trees do not fit beside the SA)
seq = bool(os.environ.get("AB_SEQ"))
nr = int(os.environ.get("AB_NR", 2_000_000))
roff, rl, _ = sas_amd.random_queries(n, nr, seed=31415, word_pos=n + 8 * nq, margin=256, len_lo=8, len_hi=257)
lens = torch.from_numpy(rl.astype(np.int64)).cuda()
qoff = torch.zeros(nr, dtype=torch.int64, device="cuda")
qoff[1:] = torch.cumsum(lens, 0)[:-1]
rsrc = torch.from_numpy(roff.astype(np.int64)).cuda()
rb = torch.empty(int(lens.sum()) + 64, dtype=torch.uint8, device="cuda")
for s0 in range(0, nr, 1 << 18):
    e0 = min(nr, s0 + (1 << 18))
    L = lens[s0:e0]
    rep_ = torch.repeat_interleave(torch.arange(e0 - s0, device="cuda"), L)
    within = torch.arange(rep_.numel(), device="cuda") - (qoff[s0:e0] - qoff[s0])[rep_]
    rb[qoff[s0]:qoff[s0] + rep_.numel()] = t[rsrc[s0:e0][rep_] + within]
ql = lens.to(torch.int32)
sa = None
idx = {}
times = {k: [] for k in kinds}
rtimes = {k: [] for k in kinds}
res, rr = {}, {}


def measure(k, ix):
    ix.time_fixed(qb, m, nq, out, algo="quad", reps=2)
    kns, _ = ix.time_fixed(qb, m, nq, out, algo="quad", reps=20)
    times[k].append(kns / 1e6)
    res[k] = out.cpu().numpy().copy()
    ro = torch.empty(nr, dtype=torch.int64, device="cuda")
    for _ in range(2):
        ix.search_batch(rb, qoff, ql, algo="quad", out=ro)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        ix.search_batch(rb, qoff, ql, algo="quad", out=ro)
    e1.record()
    torch.cuda.synchronize()
    rtimes[k].append(e0.elapsed_time(e1) / 10)
    rr[k] = ro.cpu().numpy()


reps = 1 if os.environ.get("AB_SHORT") else (2 if seq else 4)
for rep in range(reps):
    for k, v in kinds.items():
        ix = idx.get(k)
        if ix is None:
            ix = sas_amd.SaNaive.build(t, sa=sa, lcp=False, stree=False, sector=False, quad=v)
            st = ix.stats()
            print(k, "fan", st["quad_fan"], "layers", st["quad_layers"], "lds", st["quad_lds_layers"],
                  "bytes", st["quad_bytes"], flush=True)
        measure(k, ix)
        if seq:
            ix.free()
            torch.cuda.empty_cache()
        else:
            idx[k] = ix
for k in kinds:
    print(k, "quad c1 ms", " ".join(f"{x:.4f}" for x in times[k]), "min", f"{min(times[k]):.4f}",
          "| ragged ms", " ".join(f"{x:.4f}" for x in rtimes[k]), flush=True)
print("c1 identical", np.array_equal(res["rel"], res["abs"]), "ragged identical", np.array_equal(rr["rel"], rr["abs"]),
      flush=True)
