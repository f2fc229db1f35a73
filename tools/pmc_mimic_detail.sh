#!/bin/bash
# The same --pmc groups as pmc_quad_detail.sh, over the treebench replay of the quad layout.
set -o pipefail
out=$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum" \
           "SQ_BUSY_CYCLES SQ_WAIT_INST_ANY TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_STALL_MULTI_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- tools/treebench 10000000 3 1064:0.206,1064:3.5,1064:59.5,1064:1016,1064:16384 > "$out/p$i.log" 2>&1 || exit $?
done
