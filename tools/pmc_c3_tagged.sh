#!/bin/bash
# configs[3] TAGGED kernel: A/B of variant builds, then the TCC / TCP / SQ --pmc passes
# over tools/ab_c3_tagged.py (one package).  Run on the GPU box.
set -o pipefail
out=${1:-gpurun_out/c3t}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
if [ -n "$AB_PKGS" ]; then
  timeout -k 10 300 python3 tools/ab_c3_tagged.py > "$out/ab.txt" 2> "$out/ab.err" || exit $?
fi
unset AB_PKGS
export AB_NQ=${PMC_NQ:-20000000}
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$out/tcc" -o run -- python3 tools/ab_c3_tagged.py > "$out/tcc.log" 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --output-format csv -d "$out/tcp" -o run -- python3 tools/ab_c3_tagged.py > "$out/tcp.log" 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES --output-format csv -d "$out/sq" -o run -- python3 tools/ab_c3_tagged.py > "$out/sq.log" 2>&1 || exit $?
for d in tcc tcp sq; do
  f=$(ls "$out/$d"/*counter_collection.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python3 tools/pmc_summary.py "$f" k_sa_tagged "$AB_NQ" > "$out/$d.summary.txt"
done
exit 0
