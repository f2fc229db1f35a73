"""Per-access memory-side counters of randbench's shapes (tools/pmc_randbench.sh): for each
kernel, the bytes the shape reads per access, TCC_EA0_RDREQ and _32B per access, FETCH_SIZE
bytes per access and per request, and the access rate of the timed run.  This states the
request size behind the bench's traffic figures (PMC requests x 128 B) instead of assuming
it: a random read of 4..128 B is one non-32-B request, and FETCH_SIZE tallies it at 64 B, the
same half as a 128-B streaming request (MI355X_MICROARCH.md §HBM)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out = sys.argv[1]
ACC = 100_000_000
shape = {"k_stream16": ("stream16", 16), "k_rand<0>": ("rand4", 4), "k_rand<1>": ("rand8x2", 16),
         "k_rand<2>": ("rand64", 64), "k_rand<3>": ("rand128", 128), "k_rand<4>": ("rand16", 16),
         "k_rand<5>": ("rand32pair", 32), "k_rand<6>": ("rand32pair_nt", 32)}


def counters(pattern):
    f = glob.glob(os.path.join(out, pattern, "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(lambda: defaultdict(list))
    for row in csv.DictReader(open(f[0])):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


fetch, req = counters("fetch"), counters("req")
timing = {j["kernel"]: j for j in map(json.loads, open(os.path.join(out, "randbench.jsonl")))}
res = {}
for k, (name, bpa) in shape.items():
    if k not in fetch and k not in req:
        continue
    # the first dispatch is the warm-up; every dispatch moves the same count
    accesses = (1 << 32) // 16 if name == "stream16" else ACC
    f = fetch[k]["FETCH_SIZE"][-1] * 1024 / accesses if k in fetch else None
    r = req[k]
    rd = r["TCC_EA0_RDREQ_sum"][-1] / accesses
    rd32 = r["TCC_EA0_RDREQ_32B_sum"][-1] / accesses
    hit, miss = r["TCC_HIT_sum"][-1], r["TCC_MISS_sum"][-1]
    t = timing.get(name, {})
    res[name] = {"bytes_per_access": bpa, "rdreq_per_access": round(rd, 4), "rdreq_32B_per_access": round(rd32, 4),
                 "fetch_bytes_per_access": round(f, 2) if f is not None else None,
                 "fetch_bytes_per_request": round(f / rd, 2) if f and rd else None,
                 "L2_hit_rate": round(hit / (hit + miss), 4) if hit + miss else None,
                 "accesses_per_s": t.get("accesses_per_s"), "requests_per_s": (t.get("accesses_per_s") or 0) * rd}
print(json.dumps({"buffer": "4 GiB hipMalloc (>> 256 MiB Infinity Cache)", "accesses": ACC, "shapes": res}, indent=1))
