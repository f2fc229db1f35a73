"""configs[3] shape (n = 2^34 chars, ragged 8..256 queries): the rank-ordered tagged index
(SAS_BUILD_TAGGED) against bucket lines (SAS_BUILD_TAG_LINES), same queries, positions
required identical.  The two indexes are built one after the other (they do not fit
together); the lines index is built from a host copy of the text (its build peaks at the SA,
the lines and the overflow together).
    AB_N (2^34), AB_NQ (2*10^7), AB_LENS ("8-257"), AB_P (lines p, 0 = default), AB_REPS (3)"""
import os
import sys
import time

import numpy as np
import torch

root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(root, "suffix-array-searching_amd"))
import sas_amd  # noqa: E402

n = int(os.environ.get("AB_N", 1 << 34))
nq = int(os.environ.get("AB_NQ", 20_000_000))
reps = int(os.environ.get("AB_REPS", 3))
lp = int(os.environ.get("AB_P", 0))
lo_, hi_ = (int(x) for x in os.environ.get("AB_LENS", "8-257").split("-"))


def timed(idx, qb, qoff, lens, out, algo="tagged"):
    idx.search_batch(qb, qoff, lens, algo=algo, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        idx.search_batch(qb, qoff, lens, algo=algo, out=out)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


t0 = time.time()
text = sas_amd.random_string(n, seed=31415, device="cuda")
htext = text.cpu().numpy()
idx = sas_amd.SaNaive.build(text, lcp=False, tagged=True)
del text
torch.cuda.empty_cache()
print(f"tagged build {time.time() - t0:.1f} s", flush=True)
off, ln, _ = sas_amd.random_queries(n, nq, seed=31415, word_pos=n, margin=256, len_lo=lo_, len_hi=hi_)
lens = torch.from_numpy(ln.astype(np.int32)).cuda()
qoff = torch.zeros(nq, dtype=torch.int64, device="cuda")
qoff[1:] = torch.cumsum(lens.long(), 0)[:-1]
qb = torch.zeros(int(lens.sum().item()) + 64, dtype=torch.uint8, device="cuda")
idx.extract(torch.from_numpy(off.astype(np.int64)).cuda(), lens, qoff, qb)
out = torch.empty(nq, dtype=torch.int64, device="cuda")
ms = timed(idx, qb, qoff, lens, out)
ref = out.cpu()
_, pr = idx.search_batch(qb, qoff, lens, algo="tagged", probes=True)
print(f"tagged: {ms:.3f} ms per {nq} len [{lo_}, {hi_}) mean probes {pr.double().mean().item():.3f}", flush=True)
idx.free()
torch.cuda.empty_cache()
t0 = time.time()
lidx = sas_amd.SaNaive.build(htext, lcp=False, tagged=lp if lp else True, tag_lines=True)
st = lidx.stats()
print(f"lines build {time.time() - t0:.1f} s: p {st['tag_chars']}, lines {st['tag_table_bytes'] / 2**30:.1f} GiB, "
      f"overflow {st['tag_overflow_entries']} entries ({st['sa_bytes'] / 2**30:.1f} GiB), "
      f"index {st['index_bytes'] / 2**30:.1f} GiB", flush=True)
del htext
ms2 = timed(lidx, qb, qoff, lens, out)
same = bool(torch.equal(out.cpu(), ref))
_, pr2 = lidx.search_batch(qb, qoff, lens, algo="tagged", probes=True)
print(f"lines: {ms2:.3f} ms per {nq} identical={same} mean probes {pr2.double().mean().item():.3f}", flush=True)
# text slices on lines
src = torch.from_numpy(off.astype(np.int64)).cuda()
lidx.search_slices(src, lens, out=out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    lidx.search_slices(src, lens, out=out)
e1.record()
torch.cuda.synchronize()
print(f"lines slices: {e0.elapsed_time(e1) / reps:.3f} ms identical={bool(torch.equal(out.cpu(), ref))}", flush=True)
if not same:
    sys.exit(1)
