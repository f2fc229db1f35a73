"""Per-dispatch counter sums for one kernel-name substring, averaged over runs of
consecutive dispatches: usage pmc_summary.py <csv> <kernel substring> <lookups per dispatch>"""
import collections
import csv
import sys

path, name, per = sys.argv[1], sys.argv[2], float(sys.argv[3])
d = collections.OrderedDict()
for r in csv.DictReader(open(path)):
    if name not in r["Kernel_Name"]:
        continue
    e = d.setdefault(r["Dispatch_Id"], collections.Counter())
    e[r["Counter_Name"]] += float(r["Counter_Value"])
keys = list(d)
for i, k in enumerate(keys):
    print(i, " ".join(f"{c}={v / per:.3f}" for c, v in sorted(d[k].items())))
