import sys, time
sys.path.insert(0, "suffix-array-searching_amd")
import torch, sas_amd
n = (1 << 32) + 12345
t0 = time.time()
t = sas_amd.random_string(n, seed=321, device="cuda")
torch.cuda.synchronize(); t1 = time.time()
idx = sas_amd.SaNaive.build(t, lcp=True, stree=True, verify=True)
t2 = time.time()
print("gen", t1 - t0, "build", t2 - t1, idx.stats(), flush=True)
