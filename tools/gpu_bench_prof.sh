#!/bin/bash
# default bench line, then its rocprofv3 kernel statistics (tools/prof_r3.sh)
set -o pipefail
out=gpurun_out/bench
mkdir -p "$out"
timeout -k 10 900 python3 -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac']);print({k:(v.get('lookups_per_s') if isinstance(v,dict) else v) for k,v in d['configs'].items()})"
bash tools/prof_r3.sh
