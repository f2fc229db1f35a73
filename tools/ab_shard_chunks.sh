#!/bin/bash
# A/B of the sharded step in pieces (--shard-chunks) at world size 1 (GPU box).
set -o pipefail
out=gpurun_out/ab_chunks
mkdir -p "$out"
for r in 1 2; do
  for c in 1 2 4; do
    timeout -k 10 240 python3 -u bench.py --mode shard --shard-chunks $c --no-c3 --no-c4 --no-cpu --no-e2e --variants "" --steps 30 > "$out/c$c.json" 2> "$out/c$c.err" || exit $?
    python3 -c "import json;d=json.load(open('$out/c$c.json'));print('chunks',$c,round(d['ms_per_step'],4),'%.3e'%d['value'])" | tee -a "$out/summary.txt"
  done
done
