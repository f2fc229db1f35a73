"""Per-(kernel, grid, workgroup) duration summary of a rocprofv3 --kernel-trace CSV, so that
the launches of one workload (e.g. the headline's 10^7-query grid) can be told apart from
the same kernel's launches on other batch sizes (host-pipeline chunks, variants).
usage: kt_by_grid.py <run_kernel_trace.csv> <out.csv> [kernel substring ...]"""
import collections
import csv
import sys

path, out = sys.argv[1], sys.argv[2]
names = sys.argv[3:]
g = collections.defaultdict(list)
with open(path) as f:
    for r in csv.DictReader(f):
        k = r.get("Kernel_Name", "")
        if names and not any(n in k for n in names):
            continue
        grid = tuple(r.get(c, "") for c in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z", "Grid_Size") if c in r)
        wg = tuple(r.get(c, "") for c in ("Workgroup_Size_X", "Workgroup_Size") if c in r)
        g[(k, grid, wg)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Kernel_Name", "Grid", "Workgroup", "Calls", "AverageNs", "MinNs", "MaxNs", "P10Ns", "MedianNs",
                "P90Ns"])
    for (k, grid, wg), ds in sorted(g.items(), key=lambda x: -sum(x[1])):
        ds.sort()
        w.writerow([k, "x".join(x for x in grid if x), "x".join(x for x in wg if x), len(ds), sum(ds) / len(ds),
                    ds[0], ds[-1], ds[len(ds) // 10], ds[len(ds) // 2], ds[(9 * len(ds)) // 10]])
