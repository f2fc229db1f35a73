# Same-box A/B: this tree vs a build without non-temporal loads (tools/mk_variant.sh nont ...)
set -e
for r in 1 2; do
  for v in base nont; do
    pkg=""; [ "$v" != base ] && pkg=tools/_var_$v/suffix-array-searching_amd
    echo "== $v"; AB_PKG=$pkg timeout -k 10 300 python3 -u tools/ab_algos.py 2>&1 | grep "^ms"
  done
done
