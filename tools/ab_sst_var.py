"""Same-box A/B of the u32 kernels over tools/mk_variant.sh builds: the default line's lineup at
2^28 keys and 10^7 uniform queries (benchlib/sst.py's workload), the libraries under AB_PKGS
(colon-separated; 'tree' = this tree's) interleaved round-robin over AB_ROUNDS rounds.  Every
library's answers must equal the first one's.  One JSON line: {"<pkg>": {"<layout>": [ms]}}.
    AB_PKGS=tree:tools/_var_qp/suffix-array-searching_amd python3 tools/ab_sst_var.py"""
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
from benchlib.sst import SST_LINEUP, sst_layouts, sst_workload  # noqa: E402

pkgs = os.environ.get("AB_PKGS", "tree").split(":")
rounds = int(os.environ.get("AB_ROUNDS", "3"))
reps = int(os.environ.get("AB_REPS", "20"))


def load(p):
    path = os.path.join(ROOT, "suffix-array-searching_amd") if p == "tree" else os.path.join(ROOT, p)
    for k in [k for k in sys.modules if k == "sas_amd" or k.startswith("sas_amd.")]:
        del sys.modules[k]
    sys.path.insert(0, path)
    mod = importlib.import_module("sas_amd")
    sys.path.pop(0)
    return mod


mods = {p: load(p) for p in pkgs}
vals, qs = sst_workload(1 << 28, 10_000_000)
dq = torch.from_numpy(qs.view(np.int32)).cuda()
out = torch.empty(len(qs), dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream().cuda_stream
res = {p: {"source_hash": mods[p].source_hash()} for p in pkgs}
ref = {}
for name in SST_LINEUP:
    idx = {p: sst_layouts(mods[p])[name](vals) for p in pkgs}
    for rd in range(rounds):
        for p in pkgs:
            idx[p].time_query(dq, out, reps=2, stream=st)
            kns = idx[p].time_query(dq, out, reps=reps, stream=st)
            res[p].setdefault(name, []).append(round(kns / 1e6, 4))
            if name not in ref:
                ref[name] = out.clone()
            assert torch.equal(out, ref[name]), (p, name)
    for p in pkgs:
        idx[p].free()
    print(name, {p: res[p][name] for p in pkgs}, file=sys.stderr, flush=True)
print(json.dumps(res), flush=True)
