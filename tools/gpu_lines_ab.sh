#!/bin/bash
# bucket-line kernel: same-box A/B of variant builds, then its counters
set -o pipefail
out=gpurun_out/lines_ab
mkdir -p "$out"
AB_PKGS=${AB_PKGS:-suffix-array-searching_amd} timeout -k 10 600 python3 -u tools/ab_lines_var.py > "$out/ab.txt" 2> "$out/ab.err" || { tail -20 "$out/ab.err"; cat "$out/ab.txt"; exit 1; }
cat "$out/ab.txt"
[ -n "$NO_PMC" ] && exit 0
bash tools/pmc_lines.sh gpurun_out/pmc_lines
