#!/bin/bash
# Counters of the bucket-line kernel (k_sa_tagged_lines) on the configs[3] shape, separate passes.
set -o pipefail
out=${1:-gpurun_out/pmc_lines}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export AB_ROUNDS=1 AB_REPS=2
unset AB_PKGS
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$out/tcc" -o run -- python3 tools/ab_lines_var.py > "$out/tcc.log" 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --output-format csv -d "$out/tcp" -o run -- python3 tools/ab_lines_var.py > "$out/tcp.log" 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS --output-format csv -d "$out/sq" -o run -- python3 tools/ab_lines_var.py > "$out/sq.log" 2>&1 || exit $?
for d in tcc tcp sq; do
  f=$(ls "$out/$d"/*counter_collection.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python3 tools/pmc_summary.py "$f" k_sa_tagged_lines 20000000 > "$out/$d.summary.txt"
  rm -f "$f"
done
cat "$out"/*.summary.txt
exit 0
