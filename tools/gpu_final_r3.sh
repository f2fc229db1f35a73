#!/bin/bash
# Round-3 final checks on the committed tree (GPU box), in three calls:
#   a: the -m gpu suite, smoke(), the configs[3] PMC passes
#   b: the PMC passes of the headline, both configs[1] figures and QUAD
#   c: the default bench line (with the PMC summaries copied into profiles/) and its kernel statistics
set -o pipefail
out=gpurun_out/final
mkdir -p "$out"
case ${1:-a} in
  a)
    timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$out/gputest.log" 2>&1 || { tail -40 "$out/gputest.log"; exit 1; }
    tail -2 "$out/gputest.log"
    timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
    tail -1 "$out/smoke.log"
    bash tools/pmc_r3.sh c3 ;;
  b)
    bash tools/pmc_r3.sh prefix plain23 plain30 quad ;;
  c)
    bash tools/gpu_bench_prof.sh ;;
esac
