#!/bin/bash
# SQ issue/wait counters for a python command (one --pmc pass each; run on the GPU box).
# usage: tools/pmc_sq.sh <outdir> <python args...>
set -o pipefail
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM --output-format csv -d "$out/sq1" -o run -- python3 "$@" > "$out/sq1.log" 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA --output-format csv -d "$out/sq2" -o run -- python3 "$@" > "$out/sq2.log" 2>&1 || exit $?
