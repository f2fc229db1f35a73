#!/bin/bash
# One GPU call of round 6: tools/gpu_r6.sh OUTDIR STEP...  (steps run in order, the first
# failure ends the call; every step under its own time limit)
#   suite    pytest -m gpu                 smoke  __graft_entry__.smoke()
#   shard    tests/test_gpu_shard.py only  bench  the default bench line
#   quick    the c1/c2 lineup only (no c0/c3/c4/CPU/e2e/lcp_long)
#   absst    tools/ab_sst_var.py (the u32 lineup) over the tree and AB_VARS, like abbin
#   abbin    tools/ab_bin.py over the tree and the tools/_var_* builds named in AB_VARS
#   kt       the bench under rocprofv3 --kernel-trace --stats, by grid (tools/prof_r4.sh)
#   c4:W:g   tools/c4_part_probe.py W g (part g of W at the bench's share for W ranks)
#   sa       tests/test_gpu_sa.py only      lcp    the c1/c2 lineup + lcp_long + sst (no c3/c4/CPU/e2e)
#   randcal  tools/pmc_randbench.sh (random-read counter calibration)
#   pmc:k1,k2  tools/pmc_r6.sh k1 k2 (PMC / SQ passes)
set -o pipefail
out=gpurun_out/$1
shift
mkdir -p "$out"
for s in "$@"; do
    echo "[gpu_r6] $(date +%T) $s"
    case $s in
        suite) timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
                   > "$out/gputest.log" 2>&1 || exit $? ;;
        shard) timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py -m gpu -x -v --timeout 600 \
                   --timeout-method thread > "$out/shard.log" 2>&1 || exit $? ;;
        sa) timeout -k 10 900 python -u -m pytest tests/test_gpu_sa.py -m gpu -x -v --timeout 600 \
                   --timeout-method thread > "$out/sa.log" 2>&1 || exit $? ;;
        lcp) timeout -k 10 600 python -u bench.py --no-c3 --no-c4 --no-cpu --no-e2e \
                   --detail "$out/lcp_detail.json" > "$out/lcp.json" 2> "$out/lcp.err" || exit $? ;;
        randcal) bash tools/pmc_randbench.sh "$out/randcal" > "$out/randcal.log" 2>&1 || exit $? ;;
        pmc:*) bash tools/pmc_r6.sh $(echo "${s#pmc:}" | tr , " ") > "$out/pmc.log" 2>&1 || exit $? ;;
        smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $? ;;
        bench) timeout -k 10 900 python -u bench.py --detail "$out/bench_detail.json" > "$out/bench.json" \
                   2> "$out/bench.err" || exit $? ;;
        quick) timeout -k 10 300 python -u bench.py --no-c3 --no-c4 --no-cpu --no-e2e --no-lcp-long \
                   --detail "$out/quick_detail.json" > "$out/quick.json" 2> "$out/quick.err" || exit $? ;;
        abbin) AB_PKGS="tree${AB_VARS:+:}${AB_VARS}" timeout -k 10 500 python3 -u tools/ab_bin.py > "$out/ab_bin.json" \
                   2> "$out/ab_bin.err" || exit $? ;;
        abq) AB_PKGS="tree${AB_VARS:+:}${AB_VARS}" timeout -k 10 600 python3 -u tools/ab_qllcp.py > "$out/ab_qllcp.jsonl" \
                   2> "$out/ab_qllcp.err" || exit $? ;;
        c4step) timeout -k 10 300 python3 -u tools/c4_step_probe.py 30 > "$out/c4_step_probe.json" \
                   2> "$out/c4_step_probe.err" || exit $? ;;
        absst) AB_PKGS="tree${AB_VARS:+:}${AB_VARS}" timeout -k 10 500 python3 -u tools/ab_sst_var.py > "$out/ab_sst.json" \
                   2> "$out/ab_sst.err" || exit $? ;;
        kt) bash tools/prof_r5.sh "$out/prof" > "$out/prof.log" 2>&1 || exit $? ;;
        kt34) bash tools/prof_r5_c34.sh "$out/prof34" > "$out/prof34.log" 2>&1 || exit $? ;;
        c4:*) IFS=: read -r _ W g <<< "$s"
              timeout -k 10 400 python3 -u tools/c4_part_probe.py "$W" "$g" > "$out/c4probe_${W}_${g}.json" \
                  2> "$out/c4probe_${W}_${g}.err" || exit $? ;;
        *) echo "unknown step $s" >&2; exit 2 ;;
    esac
done
