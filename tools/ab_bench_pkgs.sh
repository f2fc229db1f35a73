#!/bin/bash
# Same-box A/B of library builds through bench.py itself: for each round, the tree's bench and
# the same bench.py run against tools/_var_<name> (tools/mk_variant.sh), alternating processes.
# usage: tools/ab_bench_pkgs.sh <variant name> <rounds> <out dir> -- <bench.py args>
set -o pipefail
v=$1; rounds=$2; out=$3; shift 4
root=$(cd "$(dirname "$0")/.." && pwd)
vd=$root/tools/_var_$v
for f in bench.py benchlib oracle; do [ -e "$vd/$f" ] || ln -s "$root/$f" "$vd/$f"; done
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for side in tree "$v"; do
    dir=$root; [ "$side" = tree ] || dir=$vd
    timeout -k 10 600 python3 "$dir/bench.py" "$@" --detail= > "$out/${side}_$r.json" 2> "$out/${side}_$r.err" || exit $?
    echo "[ab] round $r $side: $(tail -c 300 "$out/${side}_$r.err" | tr '\n' ' ' | tail -c 200)"
  done
done
