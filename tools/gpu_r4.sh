#!/bin/bash
# One GPU call of round 4: tools/gpu_r4.sh OUTDIR STEP...  (steps run in order, the first
# failure ends the call; every step under its own time limit)
#   suite  pytest -m gpu          smoke  __graft_entry__.smoke()
#   bench  the default bench line quick  the c1/c2 lineup only (no c0/c3/c4/CPU/e2e/lcp_long)
#   lcp    the lcp_long record (c1 lineup + lcp_long)
#   kt     the bench under rocprofv3 --kernel-trace --stats, by grid (tools/prof_r4.sh)
set -o pipefail
out=gpurun_out/$1
shift
mkdir -p "$out"
for s in "$@"; do
    case $s in
        suite) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread \
                   > "$out/gputest.log" 2>&1 || exit $? ;;
        smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $? ;;
        bench) timeout -k 10 600 python -u bench.py --detail "$out/bench_detail.json" > "$out/bench.json" \
                   2> "$out/bench.err" || exit $? ;;
        quick) timeout -k 10 300 python -u bench.py --no-c3 --no-c4 --no-cpu --no-e2e --no-lcp-long \
                   --detail "$out/quick_detail.json" > "$out/quick.json" 2> "$out/quick.err" || exit $? ;;
        lcp) timeout -k 10 300 python -u bench.py --no-c3 --no-c4 --no-cpu --no-e2e \
                   --detail "$out/lcp_detail.json" > "$out/lcp.json" 2> "$out/lcp.err" || exit $? ;;
        kt) bash tools/prof_r4.sh "$out/prof" > "$out/prof.log" 2>&1 || exit $? ;;
        *) echo "unknown step $s" >&2; exit 2 ;;
    esac
done
