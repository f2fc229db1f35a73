#!/bin/bash
# Separate rocprofv3 --pmc passes over the same bench command (run on the GPU box).
# usage: tools/pmc_pass.sh <outdir> <bench args...>
set -o pipefail
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- python3 bench.py --no-cpu "$@" > "$out/fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- python3 bench.py --no-cpu "$@" > "$out/write.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$out/req" -o run -- python3 bench.py --no-cpu "$@" > "$out/req.log" 2>&1 || exit $?
