#!/bin/bash
# Counters of DirectMap's k_sst_direct by table placement (tools/placement_probe.py: the first
# table of a process, a second beside it, ...): UTCL1 translation and L2 request counters, two
# rocprofv3 --pmc passes, summarised per group of 22 dispatches by tools/pmc_groups.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=${1:-gpurun_out/placement}
mkdir -p "$out"
timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum --output-format csv -d "$out/utcl1" -o run -- python3 tools/placement_probe.py > "$out/utcl1.log" 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --output-format csv -d "$out/tcc" -o run -- python3 tools/placement_probe.py > "$out/tcc.log" 2>&1 || exit $?
for p in utcl1 tcc; do
  python3 tools/pmc_groups.py "$(ls "$out/$p"/*counter_collection.csv | head -1)" k_sst_direct 22 > "$out/$p.summary.txt" || exit $?
  rm -rf "${out:?}/$p"
done
