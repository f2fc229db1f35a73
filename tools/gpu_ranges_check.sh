#!/bin/bash
# Range kernels: parity tests, then the default bench without the big configs (GPU box).
set -o pipefail
out=gpurun_out/ranges
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sa.py -k "occurrence_ranges" > "$out/tests.log" 2>&1 || { tail -40 "$out/tests.log"; exit 1; }
tail -3 "$out/tests.log"
timeout -k 10 400 python3 -u bench.py --no-c3 --no-c4 --no-cpu --no-e2e --variants "" > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench.json'));print(d['value'],d['ms_per_step']);print(d['occurrence_ranges'])"
