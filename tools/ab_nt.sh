# Same-box A/B of non-temporal loads / stores in the quad kernel (variants from tools/mk_variant.sh)
set -e
for r in 1 2 3; do
  for v in base nt1 nt1io nt2io nt3io; do
    pkg=""; [ "$v" != base ] && pkg=tools/_var_$v/suffix-array-searching_amd
    echo "== $v"; AB_PKG=$pkg AB_SHORT=1 timeout -k 10 200 python3 -u tools/ab_quad_rel.py 2>&1 | grep "ms"
  done
done
