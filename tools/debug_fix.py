import sys, os, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "suffix-array-searching_amd"))
import numpy as np
import sas_amd
from oracle import pyoracle as O
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from test_gpu_sa import pack
d = json.load(open(os.path.join(os.path.dirname(__file__), "..", "tests/golden/sa_definition.json")))
for c in d["cases"][:3]:
    t = np.array(c["text"], np.uint8)
    for flags in [dict(lcp=False, stree=False), dict(lcp=True, stree=True, verify=True)]:
        idx = sas_amd.SaNaive.build(t, **flags)
        qs = [q["q"] for q in c["queries"]]
        buf, off, lens = pack(qs)
        exp = np.array([q["pos"] for q in c["queries"]], np.uint64)
        got, pr = idx.search_batch(buf, off, lens, algo="plain", probes=True)
        got2 = idx.search([np.array(q, np.uint8) for q in qs], algo="plain")
        print(c["name"], flags, "batch ok" if np.array_equal(got, exp) else "batch BAD", "search ok" if np.array_equal(got2, exp) else "search BAD")
        if not np.array_equal(got, exp):
            print(" lens", lens.tolist()[:20], "off", off.tolist()[:20], buf.dtype, buf.shape)
            print(" got", got.tolist()[:20]); print(" exp", exp.tolist()[:20]); print(" probes", pr.tolist()[:20])
