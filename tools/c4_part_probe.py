"""Rehearse one rank of the driver's 8-GPU configs[4] record on one GPU: a text of W x share
chars, this rank's part built as the bench builds it (sas_build_part_gen: the text generated
straight into the packed words; the two-suffix inline table at p = 16 over the part's own key
interval; the LDS pivot levels only), setup time, index bytes, the device memory left, and the
local PREFIX lookup of 10^7 packed len-32 queries (the part's share of a step).  share_log2
defaults to the bench's choice for W ranks (bench.c4_share_for).
usage: c4_part_probe.py [parts] [part] [share_log2]   (GPU box)"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "suffix-array-searching_amd"))
import bench  # noqa: E402
import sas_amd  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
g = int(sys.argv[2]) if len(sys.argv) > 2 else W - 1
torch.cuda.init()
share = (1 << int(sys.argv[3])) if len(sys.argv) > 3 else bench.c4_share_for(W, torch.cuda.mem_get_info()[1])
n, nq, m = share * W, 10_000_000, 32
t0 = time.perf_counter()
idx = sas_amd.SaNaive.build_part_gen(n, seed=bench.SEED + 1, part=g, parts=W, lcp=False, stree=False, sector=False,
                                     quad=True, llcp=False, prefix=16, prefix_inline=2,
                                     top2_levels=bench.TOP_LDS_LEVELS)
torch.cuda.synchronize()
t1 = time.perf_counter()
free, total = torch.cuda.mem_get_info()
st = idx.stats()
off = torch.from_numpy(bench.rank_query_offsets(n, nq, m, g).astype(np.int64)).cuda()
q = torch.empty(nq * m, dtype=torch.uint8, device="cuda")
idx.extract(off, torch.full((nq,), m, dtype=torch.int32, device="cuda"),
            torch.arange(nq, device="cuda", dtype=torch.int64) * m, q)
w = sas_amd.SaNaive.pack_queries(q, m)
out = torch.empty(nq, dtype=torch.int64, device="cuda")
t = bench.launch_times(torch, lambda: idx.search_packed(w, m, out=out), 10, 3, torch.cuda.current_stream())
print(json.dumps({"parts": W, "part": g, "n": n, "build_part_gen_s": round(t1 - t0, 2),
                  "sa_entries": st["sa_entries"], "rank_lo": st["rank_lo"], "sa_width": st["sa_width"],
                  "prefix_chars": st["prefix_chars"], "prefix_bytes": st["prefix_bytes"],
                  "prefix_key_lo": st["prefix_key_lo"], "prefix_entries": st["prefix_entries"],
                  "prefix_key_fraction": round(st["prefix_entries"] / (4 ** st["prefix_chars"] + 1), 4),
                  "estimate_bytes": bench.c4_part_bytes(share, W), "share": share,
                  "index_bytes": st["index_bytes"], "free_GiB_after_build": round(free / 2**30, 1),
                  "total_GiB": round(total / 2**30, 1),
                  "local_prefix_packed_ms": round(t["mean_ms"], 4),
                  "note": "local lookups of this rank's own queries (most lie in other parts: their answers are "
                          "next_pos or SA[lo] inside; the time is the kernel's)"}), flush=True)
