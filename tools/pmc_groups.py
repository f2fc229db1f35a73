"""Mean of each counter over consecutive groups of G dispatches of one kernel in a rocprofv3
counter_collection.csv: python3 tools/pmc_groups.py run_counter_collection.csv KERNEL G"""
import csv
import sys
from collections import defaultdict

path, kern, g = sys.argv[1], sys.argv[2], int(sys.argv[3])
vals = defaultdict(lambda: defaultdict(float))
for row in csv.DictReader(open(path)):
    if kern in row["Kernel_Name"]:
        vals[int(row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
ids = sorted(vals)
names = sorted({c for d in vals.values() for c in d})
for s in range(0, len(ids), g):
    grp = ids[s:s + g]
    print(f"group {s // g} dispatches {grp[0]}..{grp[-1]}",
          " ".join(f"{c}={sum(vals[i][c] for i in grp) / len(grp):.4g}" for c in names))
