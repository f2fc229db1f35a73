"""Does where a large random-access table lands in HBM change its lookup rate?  DirectMap
(9.6 GB table at 2^28 keys, 10^7 uniform queries) timed (a) built first in a fresh process,
(b) a second copy beside it, (c) rebuilt after the u32 lineup's other layouts were built and
freed (the bench's order), (d) again after that.  One JSON line {"case": ms}."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "suffix-array-searching_amd"))
import sas_amd  # noqa: E402
from benchlib.sst import SST_LINEUP, sst_layouts, sst_workload  # noqa: E402

vals, qs = sst_workload(1 << 28, 10_000_000)
dq = torch.from_numpy(qs.view(np.int32)).cuda()
out = torch.empty(len(qs), dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream().cuda_stream
mk = sst_layouts(sas_amd)
res = {}


def t(ix, name):
    ix.time_query(dq, out, reps=2, stream=st)
    res[name] = round(ix.time_query(dq, out, reps=20, stream=st) / 1e6, 4)
    print(name, res[name], file=sys.stderr, flush=True)


ballast_gb = float(os.environ.get("PROBE_BALLAST_GB", "0"))
ballast = torch.empty(int(ballast_gb * 2**30), dtype=torch.uint8, device="cuda") if ballast_gb else None
a = mk["DirectMap"](vals)
t(a, "a_fresh")
b = mk["DirectMap"](vals)
t(b, "b_second")
t(a, "a_again")
a.free()
b.free()
for name in SST_LINEUP:
    if name not in ("DirectMap", "SortedVec"):
        ix = mk[name](vals)
        t(ix, name)
        ix.free()
c = mk["DirectMap"](vals)
t(c, "c_after_lineup")
d = mk["DirectMap"](vals)
t(d, "d_second_after_lineup")
c.free()
d.free()
print(json.dumps({"ballast_gb": ballast_gb, "mode": os.environ.get("SST_ALLOC_MODE", "0"), **res}), flush=True)
