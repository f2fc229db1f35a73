#!/bin/bash
# Routing: parity tests, then the send-side timing per part count (GPU box).
set -o pipefail
out=gpurun_out/route
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_shard.py tests/test_gpu_sa.py -k "route or shard" > "$out/tests.log" 2>&1 || { tail -40 "$out/tests.log"; exit 1; }
tail -3 "$out/tests.log"
timeout -k 10 300 python3 -u tools/route_bench.py > "$out/route_bench.jsonl" 2> "$out/route_bench.err" || { tail -20 "$out/route_bench.err"; exit 1; }
cut -c1-120 "$out/route_bench.jsonl"
