import sys, os, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "suffix-array-searching_amd"))
import numpy as np
import sas_amd
from oracle import pyoracle as O
t = np.zeros(100, np.uint8)
idx = sas_amd.SaNaive.build(t)
sa = O.build_sa(t)
tp = O.padded(t)
for maxlen in (20, 40, 70, 105, 300):
    qs = [np.zeros(L, np.uint8) for L in (5, 10, 17)] + [np.full(maxlen, 3, np.uint8)]
    for algo in ("plain", "lcp", "stree"):
        got = idx.search(qs, algo=algo)
        exp = [O.search_one(tp, 100, sa, q)[0] for q in qs]
        print(maxlen, algo, got.tolist(), exp)
