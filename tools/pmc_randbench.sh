#!/bin/bash
# Calibrate the memory-side counters on random reads of known shapes (GPU box): randbench's
# 4-B, 16-B, 32-B (lane pair), 64-B and 128-B random reads over a 4 GiB buffer (>> the 256 MiB
# Infinity Cache) and a 16-B/lane stream, 10^8 accesses each, in separate rocprofv3 --pmc
# passes (FETCH_SIZE; TCC_EA0_RDREQ + _32B + hit/miss), then per-access counters
# (tools/randbench_calib.py).  usage: tools/pmc_randbench.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/randcal}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 120 rocprofv3 -L > "$out/counters_avail.txt" 2>&1 || true
args="4096 100000000 2 0 0x7f"
timeout -k 10 120 ./tools/randbench $args > "$out/randbench.jsonl" 2> "$out/randbench.err" || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- ./tools/randbench $args \
    > "$out/fetch.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --output-format csv \
    -d "$out/req" -o run -- ./tools/randbench $args > "$out/req.log" 2>&1 || exit $?
python3 tools/randbench_calib.py "$out" > "$out/randbench_calibration.json" || exit $?
find "$out/fetch" "$out/req" -name '*.csv' ! -name '*counter_collection*' -delete
