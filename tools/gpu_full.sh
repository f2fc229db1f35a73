#!/bin/bash
# Full GPU check (GPU box): the -m gpu suite, smoke(), and the default bench line.
set -o pipefail
out=gpurun_out/full
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > "$out/gputest.log" 2>&1 || { tail -40 "$out/gputest.log"; exit 1; }
tail -2 "$out/gputest.log"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
tail -2 "$out/smoke.log"
timeout -k 10 900 python3 -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac']);print({k:(v.get('lookups_per_s') if isinstance(v,dict) else v) for k,v in d['configs'].items()});print(d['cpu_baseline']);print(d['occurrence_ranges']['kernel_ms'])"
