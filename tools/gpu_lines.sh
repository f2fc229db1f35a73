#!/bin/bash
# bucket-line index on the GPU box: its parity tests, then the configs[3] A/B against TAGGED
set -o pipefail
out=gpurun_out/lines
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_gpu_tagged.py -x -v --timeout 300 --timeout-method thread > "$out/test.log" 2>&1 || { tail -30 "$out/test.log"; exit 1; }
tail -3 "$out/test.log"
timeout -k 10 600 python3 -u tools/ab_c3_lines.py > "$out/ab.txt" 2> "$out/ab.err" || { tail -20 "$out/ab.err"; cat "$out/ab.txt"; exit 1; }
cat "$out/ab.txt"
