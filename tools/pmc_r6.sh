#!/bin/bash
# Round-6 PMC passes (GPU box): separate rocprofv3 --pmc runs (FETCH_SIZE; WRITE_SIZE;
# TCC_EA0_RDREQ + 32B + hit/miss) over bench.py for each record whose traffic bench.py
# reports, summarised into gpurun_out/pmc_r6/pmc_<key>.json stamped with the library's source
# hash (copy them into profiles/ to have bench.py attach them); `sq_<key>`: the SQ issue / wait
# counters of that record's kernel (two passes, tools/pmc_sq.sh).
# usage: tools/pmc_r6.sh [keys...]
#   keys: prefix plain27 plain31 quad quad_llcp stree stree_llcp sector llcp c3 c3tagged
#         sst_stree sst_pmap16 sst_pmap20 sst_direct sst_sorted      sq_<key> (SQ passes)
#         ta_<key>: one pass of SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD TA_BUSY_avr TA_BUSY_max
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/pmc_r6
mkdir -p "$out"
keys=${*:-prefix plain27 plain31 quad quad_llcp stree stree_llcp sector llcp c3 sst_stree sst_pmap16 sst_direct}
base="--no-cpu --no-c3 --no-c4 --no-sst --no-e2e --no-lcp-long --variants= --c1-deep-levels 0 --steps 3 --warmup 1 --detail="
sst="--workload sst --no-cpu --steps 3 --warmup 1 --sst-layouts"
K=268435456
for k in $keys; do
  sq=0
  case $k in
    sq_*) sq=1; k=${k#sq_} ;;
    ta_*) sq=2; k=${k#ta_} ;;
  esac
  case $k in
    prefix)  args="$base --algo prefix"; kern=k_sa_prefix2; nq=10000000; name=prefix16d_n1073741824_q10000000_m32 ;;
    plain27) args="$base --algo plain"; kern=k_sa_binary; nq=10000000; name=plain_n1073741824_q10000000_m32_t27 ;;
    plain31) args="$base --algo plain --top2-levels 30"; kern=k_sa_binary; nq=10000000; name=plain_n1073741824_q10000000_m32_t31 ;;
    plain)   args="$base --algo plain"; kern=k_sa_binary; nq=10000000; name=plain_n1073741824_q10000000_m32_t27 ;;
    quad)    args="$base --algo quad"; kern=k_sa_quad; nq=10000000; name=quad_n1073741824_q10000000_m32 ;;
    quad_llcp) args="$base --algo quad_llcp"; kern=k_sa_quad; nq=10000000; name=quad_llcp_n1073741824_q10000000_m32 ;;
    stree)   args="$base --algo stree"; kern=k_sa_stree; nq=10000000; name=stree_n1073741824_q10000000_m32 ;;
    stree_llcp) args="$base --algo stree_llcp"; kern=k_sa_stree4x; nq=10000000; name=stree_llcp_n1073741824_q10000000_m32 ;;
    sector)  args="$base --algo sector"; kern=k_sa_sector; nq=10000000; name=sector_n1073741824_q10000000_m32 ;;
    llcp)    args="$base --algo llcp"; kern=k_sa_binary; nq=10000000; name=llcp_n1073741824_q10000000_m32 ;;
    c3)      args="--workload c3 --c3-steps 2 --warmup 1 --c3-no-cross --detail="; kern=k_sa_tagged_lines; nq=100000000; name=c3_tagged_lines_n17179869184_q100000000 ;;
    c3tagged) args="--workload c3 --c3-steps 2 --warmup 1 --c3-no-cross --c3-layout tagged --detail="; kern=k_sa_tagged; nq=100000000; name=c3_tagged_n17179869184_q100000000 ;;
    sst_stree)  args="$sst STree16_left_max"; kern=k_sst_stree4; nq=10000000; name=sst_STree16_left_max_k${K}_q10000000 ;;
    sst_pmap16) args="$sst PartitionedSTree16M_b16"; kern=k_sst_pmap4; nq=10000000; name=sst_PartitionedSTree16M_b16_k${K}_q10000000 ;;
    sst_pmap20) args="$sst PartitionedSTree16M_b20"; kern=k_sst_pmap4; nq=10000000; name=sst_PartitionedSTree16M_b20_k${K}_q10000000 ;;
    sst_direct) args="$sst DirectMap"; kern=k_sst_direct; nq=10000000; name=sst_DirectMap_k${K}_q10000000 ;;
    sst_sorted) args="$sst SortedVec"; kern=k_sst_sorted; nq=10000000; name=sst_SortedVec_k${K}_q10000000 ;;
    *) echo "unknown key $k"; exit 2 ;;
  esac
  d=$out/$k
  mkdir -p "$d"
  if [ $sq = 2 ]; then
    echo "[pmc_r6] ta $k: $args"
    timeout -s KILL 420 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY TA_BUSY_avr TA_BUSY_max TA_ADDR_STALLED_BY_TC_CYCLES_sum --output-format csv -d "$d/ta/sq_ta" -o run -- python3 bench.py $args > "$d/ta.log" 2>&1 || exit $?
    python3 tools/sq_to_json.py "$d/ta" "$kern" > "$out/ta_$k.json" || exit $?
    find "$d/ta" -name "*.csv" -delete
    continue
  fi
  if [ $sq = 1 ]; then
    echo "[pmc_r6] sq $k: $args"
    bash tools/pmc_sq.sh "$d/sq" bench.py $args || exit $?
    python3 tools/sq_to_json.py "$d/sq" "$kern" > "$out/sq_$k.json" || exit $?
    find "$d/sq" -name "*.csv" -delete
    continue
  fi
  echo "[pmc_r6] $k: $args"
  timeout -s KILL 420 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$d/fetch" -o run -- python3 bench.py $args > "$d/fetch.log" 2>&1 || exit $?
  timeout -s KILL 420 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$d/write" -o run -- python3 bench.py $args > "$d/write.log" 2>&1 || exit $?
  timeout -s KILL 420 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$d/req" -o run -- python3 bench.py $args > "$d/req.log" 2>&1 || exit $?
  f=$(ls "$d"/fetch/*counter_collection.csv | head -1)
  w=$(ls "$d"/write/*counter_collection.csv | head -1)
  r=$(ls "$d"/req/*counter_collection.csv | head -1)
  python3 tools/pmc_to_json.py --kernel "$kern" --nq $nq --fetch "$f" --write "$w" --req "$r" --out "$out/pmc_$name.json" || exit $?
  rm -rf "$d/fetch" "$d/write" "$d/req"  # the per-dispatch CSVs: too big to bring back
done
exit 0
