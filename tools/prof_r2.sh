#!/bin/bash
# Round-2 profiles (run on the GPU box): rocprofv3 kernel stats of the default bench (without
# its host-buffer pass, whose 2^19-query chunks launch the headline kernel on the same grid
# and would mix into its average), and the
# separate --pmc passes (FETCH_SIZE, WRITE_SIZE, TCC_EA0_RDREQ) of the configs[3] TAGGED run
# and of the configs[1] PLAIN run, summarised into profiles/pmc_*.json for bench.py.
set -o pipefail
out=gpurun_out/prof
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
what=${1:-all}
if [ "$what" = all ] || [ "$what" = kt ]; then
  # without the prefix_packed variant and configs[4] (both launch k_sa_prefix2 on the
  # headline's grid with packed words), so that grid's average is the headline's alone
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- python3 bench.py --no-e2e --no-c4 --variants plain,plain_range,lcp,llcp,stree,sector,quad,inline,interp,interp_range > "$out/kt_bench.json" 2> "$out/kt_bench.err" || exit $?
  python3 tools/kt_by_grid.py "$out/kt/run_kernel_trace.csv" "$out/kt/kernel_stats_by_grid.csv" k_sa_ || exit $?
  find "$out/kt" -name '*kernel_trace.csv' -delete  # per-dispatch rows: too big to bring back
fi
if [ "$what" = all ] || [ "$what" = c3 ]; then
  bash tools/pmc_pass.sh "$out/c3" --workload c3 --algo tagged --c3-steps 2 --warmup 1 || exit $?
  python3 tools/pmc_to_json.py --kernel k_sa_tagged --nq 100000000 --fetch "$out/c3/fetch/run_counter_collection.csv" \
    --write "$out/c3/write/run_counter_collection.csv" --req "$out/c3/req/run_counter_collection.csv" \
    --out "$out/pmc_c3_tagged_n17179869184_q100000000.json" || exit $?
  rm -rf "$out/c3/fetch" "$out/c3/write" "$out/c3/req"
fi
if [ "$what" = all ] || [ "$what" = plain ]; then
  bash tools/pmc_pass.sh "$out/plain" --algo plain --variants "" --no-c3 --no-e2e --steps 3 --warmup 1 || exit $?
  python3 tools/pmc_to_json.py --kernel k_sa_binary --nq 10000000 --fetch "$out/plain/fetch/run_counter_collection.csv" \
    --write "$out/plain/write/run_counter_collection.csv" --req "$out/plain/req/run_counter_collection.csv" \
    --out "$out/pmc_plain_n1073741824_q10000000_m32.json" || exit $?
  rm -rf "$out/plain/fetch" "$out/plain/write" "$out/plain/req"
fi
exit 0
