"""Same-box A/B of the u32 S-tree kernels: this tree's library vs tools/_old."""
import sys, os
which = sys.argv[1]
root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_old" if which == "old" else "..")
sys.path.insert(0, os.path.join(root, "suffix-array-searching_amd"))
import numpy as np
import torch
import sas_amd
rng = np.random.default_rng(31415)
nk, nq = 1 << 28, 10_000_000
vals = rng.integers(0, 0x7FFFFFFF, nk, dtype=np.uint64).astype(np.uint32)
vals[0] = 0x7FFFFFFF
vals.sort()
qs = rng.integers(0, 0x7FFFFFFF, nq, dtype=np.uint64).astype(np.uint32)
dq = torch.from_numpy(qs.view(np.int32)).cuda()
out = torch.empty(nq, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream().cuda_stream
for name, mk in [("STree16", lambda: sas_amd.STree16.new(vals)),
                 ("STree16_left_max", lambda: sas_amd.STree16.new_params(vals, True, False, False)),
                 ("STree15", lambda: sas_amd.STree15.new(vals)),
                 ("PartitionedSTree16M_b20", lambda: sas_amd.PartitionedSTree16M.new(vals, 20))]:
    idx = mk()
    idx.time_query(dq, out, reps=3, stream=st)
    kns = idx.time_query(dq, out, reps=20, stream=st)
    np.save(f"/tmp/abs_{which}_{name}.npy", out.cpu().numpy())
    print(which, name, f"{kns / 1e6:.4f} ms", flush=True)
    idx.free()
