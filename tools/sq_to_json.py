"""The SQ issue / wait counters of one kernel (tools/pmc_sq.sh's two passes) as one JSON: the
median over the kernel's dispatches of each counter, and the ratios that say whether a
latency-bound kernel waits on memory (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES), issues
(SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES) or is limited by VMEM issue.
usage: sq_to_json.py <pmc_sq outdir> <kernel name>"""
import glob
import json
import os
import re
import sys
from collections import defaultdict

out, kernel = sys.argv[1], sys.argv[2]
pat = re.compile(r"(^|[^\w])" + re.escape(kernel) + r"\s*[<(]")
vals = defaultdict(lambda: defaultdict(float))
for f in glob.glob(os.path.join(out, "sq*", "**", "*counter_collection.csv"), recursive=True):
    import csv
    for row in csv.DictReader(open(f)):
        if pat.search(row.get("Kernel_Name", "")):
            vals[(os.path.basename(os.path.dirname(f)), row["Dispatch_Id"])][row["Counter_Name"]] += \
                float(row["Counter_Value"])
per = defaultdict(list)
for d in vals.values():
    for c, v in d.items():
        per[c].append(v)
med = {c: sorted(v)[len(v) // 2] for c, v in per.items()}
res = {"kernel": kernel, "dispatches": {c: len(v) for c, v in per.items()}, "median": med}
wc = med.get("SQ_WAVE_CYCLES")
if wc:
    for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM",
              "SQ_ACTIVE_INST_LDS"):
        if c in med:
            res[c + "_per_wave_cycle"] = med[c] / wc
print(json.dumps(res, indent=1))
