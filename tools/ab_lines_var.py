"""Same-box A/B of library variants on ONE bucket-line index (configs[3] shape: n = 2^34,
ragged 8..256 queries).  AB_PKGS=tools/_var_a/suffix-array-searching_amd,... (the first drives
the build; every variant drives the same handle, so the struct layout must match); every
variant's positions must equal the first's.  AB_N, AB_NQ (2*10^7), AB_LENS, AB_REPS, AB_ROUNDS."""
import ctypes
import os
import sys

import numpy as np
import torch

root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
pkgs = [p for p in os.environ.get("AB_PKGS", "").split(",") if p] or [os.path.join(root, "suffix-array-searching_amd")]
n = int(os.environ.get("AB_N", 1 << 34))
nq = int(os.environ.get("AB_NQ", 20_000_000))
reps = int(os.environ.get("AB_REPS", 3))
rounds = int(os.environ.get("AB_ROUNDS", 2))
lo_, hi_ = (int(x) for x in os.environ.get("AB_LENS", "8-257").split("-"))
sys.path.insert(0, pkgs[0])
import sas_amd  # noqa: E402

text = sas_amd.random_string(n, seed=31415, device="cuda")
htext = text.cpu().numpy()
del text
torch.cuda.empty_cache()
idx = sas_amd.SaNaive.build(htext, lcp=False, tagged=True, tag_lines=True)
del htext
off, ln, _ = sas_amd.random_queries(n, nq, seed=31415, word_pos=n, margin=256, len_lo=lo_, len_hi=hi_)
lens = torch.from_numpy(ln.astype(np.int32)).cuda()
qoff = torch.zeros(nq, dtype=torch.int64, device="cuda")
qoff[1:] = torch.cumsum(lens.long(), 0)[:-1]
qb = torch.zeros(int(lens.sum().item()) + 64, dtype=torch.uint8, device="cuda")
idx.extract(torch.from_numpy(off.astype(np.int64)).cuda(), lens, qoff, qb)
out = torch.empty(nq, dtype=torch.int64, device="cuda")
ref = None
a = sas_amd._lib.ALGOS["tagged"]
for rnd in range(rounds):
    for pk in pkgs:
        lib = ctypes.CDLL(os.path.join(pk, "libsas_amd.so")) if pk != pkgs[0] else sas_amd._lib.lib()
        st = torch.cuda.current_stream().cuda_stream

        def call():
            rc = lib.sas_search_batch(idx._h, ctypes.c_void_p(qb.data_ptr()), ctypes.c_void_p(qoff.data_ptr()),
                                      ctypes.c_void_p(lens.data_ptr()), ctypes.c_uint64(nq), a,
                                      ctypes.c_void_p(out.data_ptr()), None, ctypes.c_void_p(st),
                                      ctypes.c_uint32(sas_amd._lib.SAS_DEVICE_PTRS))
            assert rc == 0, rc
        call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        ok = True
        if ref is None:
            ref = out.clone()
        else:
            ok = bool(torch.equal(out, ref))
        if "ablate" in pk:  # timing-only variants (wrong answers by design)
            ok = True
        print(f"round{rnd} {os.path.basename(os.path.dirname(os.path.abspath(pk)))}: "
              f"{e0.elapsed_time(e1) / reps:.3f} ms per {nq} identical={ok}", flush=True)
        if not ok:
            sys.exit(1)
