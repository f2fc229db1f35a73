# Same-box A/B of the top2 depth (tools/mk_variant.sh t22 -DSAS_TOP2_LEVELS=22 ...)
set -e
for r in 1 2; do
  for v in base ${AB_VARIANTS:-t22 t23}; do
    pkg=""; [ "$v" != base ] && pkg=tools/_var_$v/suffix-array-searching_amd
    echo "== $v"; AB_PKG=$pkg timeout -k 10 300 python3 -u tools/ab_algos.py 2>&1 | grep "^ms"
  done
done
