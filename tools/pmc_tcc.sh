#!/bin/bash
# L2 / fabric request counters for a python command (one --pmc pass; run on the GPU box).
# usage: tools/pmc_tcc.sh <outdir> <python args...>
set -o pipefail
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$out/tcc" -o run -- python3 "$@" > "$out/tcc.log" 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --output-format csv -d "$out/tcp" -o run -- python3 "$@" > "$out/tcp.log" 2>&1 || exit $?
