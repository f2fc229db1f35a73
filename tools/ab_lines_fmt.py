"""configs[3] shape (n = 2^34, ragged 8..256 queries) on ONE bucket-line library: build the
line index from a host copy of the text, time TAGGED on byte queries and text slices, save
the positions.  Run once per library (AB_PKG = a package dir, e.g. tools/_var_old/...) on
the same box, then compare the saved positions (AB_OUT) across runs: line formats differ, so
the two libraries cannot share one index.
    AB_PKG, AB_OUT (/tmp/ab_lines_<tag>.npy), AB_TAG, AB_N (2^34), AB_NQ (2*10^7),
    AB_LENS ("8-257"), AB_REPS (3), AB_ROUNDS (3)"""
import os
import sys
import time

import numpy as np
import torch

root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
pkg = os.environ.get("AB_PKG") or os.path.join(root, "suffix-array-searching_amd")
sys.path.insert(0, pkg)
import sas_amd  # noqa: E402

tag = os.environ.get("AB_TAG", "new")
n = int(os.environ.get("AB_N", 1 << 34))
nq = int(os.environ.get("AB_NQ", 20_000_000))
reps = int(os.environ.get("AB_REPS", 3))
rounds = int(os.environ.get("AB_ROUNDS", 3))
lo_, hi_ = (int(x) for x in os.environ.get("AB_LENS", "8-257").split("-"))

t0 = time.time()
htext = sas_amd.random_string(n, seed=31415, device="cuda").cpu().numpy()
torch.cuda.empty_cache()
idx = sas_amd.SaNaive.build(htext, lcp=False, tagged=True, tag_lines=True)
del htext
st = idx.stats()
print(f"[{tag}] lines build {time.time() - t0:.1f} s: p {st['tag_chars']}, slots {st['tag_line_slots']}, "
      f"tables {st['tag_table_bytes'] / 2**30:.1f} GiB, overflow {st['tag_overflow_entries']} entries, "
      f"index {st['index_bytes'] / 2**30:.1f} GiB", flush=True)
off, ln, _ = sas_amd.random_queries(n, nq, seed=31415, word_pos=n, margin=256, len_lo=lo_, len_hi=hi_)
lens = torch.from_numpy(ln.astype(np.int32)).cuda()
qoff = torch.zeros(nq, dtype=torch.int64, device="cuda")
qoff[1:] = torch.cumsum(lens.long(), 0)[:-1]
qb = torch.zeros(int(lens.sum().item()) + 64, dtype=torch.uint8, device="cuda")
idx.extract(torch.from_numpy(off.astype(np.int64)).cuda(), lens, qoff, qb)
src = torch.from_numpy(off.astype(np.int64)).cuda()
out = torch.empty(nq, dtype=torch.int64, device="cuda")


def timed(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for r in range(rounds):
    ms = timed(lambda: idx.search_batch(qb, qoff, lens, algo="tagged", out=out))
    ms_s = timed(lambda: idx.search_slices(src, lens, out=out))
    print(f"[{tag}] round{r}: bytes {ms:.3f} ms, slices {ms_s:.3f} ms per {nq}", flush=True)
idx.search_batch(qb, qoff, lens, algo="tagged", out=out)
torch.cuda.synchronize()
pos = out.cpu().numpy()
np.save(os.environ.get("AB_OUT", f"/tmp/ab_lines_{tag}.npy"), pos)
# every answer is an occurrence (positive queries): its text equals the query
k = np.random.default_rng(1).choice(nq, 20000, replace=False)
chk = torch.zeros(int(ln[k].sum()) + 64, dtype=torch.uint8, device="cuda")
ko = np.zeros(len(k), np.int64)
ko[1:] = np.cumsum(ln[k].astype(np.int64))[:-1]
idx.extract(torch.from_numpy(pos[k].astype(np.int64)).cuda(), lens[torch.from_numpy(k).cuda()],
            torch.from_numpy(ko).cuda(), chk)
qk = torch.zeros_like(chk)
idx.extract(src[torch.from_numpy(k).cuda()], lens[torch.from_numpy(k).cuda()], torch.from_numpy(ko).cuda(), qk)
print(f"[{tag}] 20000 sampled answers are occurrences: {bool(torch.equal(chk, qk))}", flush=True)
