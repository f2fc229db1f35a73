#!/bin/bash
# L2->fabric requests and SQ counters of the LCP-skipping kernels on the lcp_long shapes
# (tools/ab_qllcp.py under two rocprofv3 --pmc passes), summarised per kernel into
# gpurun_out/pmc_rep$PMC_TAG/summary.txt.  AB_TEXTS / AB_MS / AB_ALGOS / AB_PKGS as ab_qllcp.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/pmc_rep${PMC_TAG:-}
mkdir -p $out
export OUT=$out
export AB_TEXTS=${AB_TEXTS:-repetitive} AB_MS=${AB_MS:-64,256} AB_ALGOS=${AB_ALGOS:-stree_llcp,quad_llcp,llcp} AB_ROUNDS=1 AB_REPS=3
timeout -s KILL 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $out/req -o run -- python3 tools/ab_qllcp.py > $out/req.log 2>&1 || exit $?
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d $out/sq -o run -- python3 tools/ab_qllcp.py > $out/sq.log 2>&1 || exit $?
python3 - <<'PY' > $out/summary.txt
import csv, glob, collections, statistics, os
for d in ("req", "sq"):
    f = glob.glob(f"{os.environ['OUT']}/{d}/**/*counter_collection.csv", recursive=True)[0]
    disp = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if not any(s in k for s in ("llcp", "binary", "stree4x")):
            continue
        disp[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = k
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for i, cs in disp.items():
        for c, v in cs.items():
            acc[names[i]][c].append(v)
    for k, cs in sorted(acc.items()):
        print(d, k[:70], {c: round(statistics.median(v)) for c, v in cs.items()}, "n=%d" % len(next(iter(cs.values()))))
PY
cat $out/summary.txt
find $out -name "*.csv" -size +2M -delete
