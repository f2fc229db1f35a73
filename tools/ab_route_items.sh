#!/bin/bash
# A/B of the one-pass route+scatter's queries per thread (SAS_ROUTE_ITEMS) on the ws = 1
# sharded step (run on the GPU box); one bench line per run, alternating.
set -o pipefail
out=gpurun_out/ab_route_items
mkdir -p "$out"
for it in 8 4 2 8 4 2; do
  SAS_ROUTE_ITEMS=$it timeout -k 10 240 python3 -u bench.py --mode shard --no-c3 --no-c4 --no-cpu --no-e2e --variants "" --steps 30 > "$out/items$it.json" 2> "$out/items$it.err" || exit $?
  python3 -c "import json,sys;d=json.load(open('$out/items$it.json'));print('items',$it,round(d['ms_per_step'],4),'%.3e'%d['value'])" | tee -a "$out/summary.txt"
done
