"""Host-pointer search timing (the bench's e2e_host pass) with the pipeline's phase trace:
SAS_STAGE_TRACE=1 python3 tools/e2e_host.py [algo]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "suffix-array-searching_amd"))
import sas_amd  # noqa: E402

algo = sys.argv[1] if len(sys.argv) > 1 else "prefix"
n, nq, m = 1 << 30, 10_000_000, 32
t = sas_amd.random_string(n, seed=31415, device="cuda")
idx = sas_amd.SaNaive.build(t, lcp=False, stree=False, sector=False, llcp=False, prefix=16, prefix_inline=2)
off, _, _ = sas_amd.random_queries(n, nq, seed=31415, word_pos=n, margin=200, len_lo=m, len_hi=m + 1)
ot = torch.from_numpy(off.astype(np.int64)).cuda()
qb = t[(ot[:, None] + torch.arange(m, device="cuda")[None, :]).reshape(-1)].cpu().numpy()
dev = idx.search_fixed(torch.from_numpy(qb).cuda(), m, algo=algo)
torch.cuda.synchronize()
ref = dev.cpu().numpy().astype(np.uint64)
for r in range(4):
    t0 = time.perf_counter()
    got = idx.search_fixed(qb, m, algo=algo)
    dt = time.perf_counter() - t0
    print(f"host call {r}: {dt * 1e3:.2f} ms, identical={np.array_equal(got, ref)}", flush=True)
t0 = time.perf_counter()
z = np.zeros(nq, np.uint64)
z[:] = 1
print(f"np.zeros + first touch of {nq * 8 >> 20} MiB: {(time.perf_counter() - t0) * 1e3:.2f} ms")
t0 = time.perf_counter()
c = qb.copy()
print(f"numpy copy of {len(qb) >> 20} MiB: {(time.perf_counter() - t0) * 1e3:.2f} ms")
