#!/bin/bash
# Price configs[3] layouts with tools/treebench (GPU box): the tagged chain as it is
# (bucket word 8 B of 32 GiB, window 16 B of 128 GiB, text 32 B of 4 GiB, per lane) against
# a bucket-line table (the bucket's header + first entries in one 128-B line of a 128 GiB
# table read by an 8-lane group, or a 64-B line by a 4-lane group), each lookup streaming
# 132 query bytes as wave-contiguous spans.
set -o pipefail
out=${1:-gpurun_out/tb_c3}
mkdir -p "$out"
tb=tools/treebench
N=${TB_N:-20000000}
run() { echo "== $*" >> "$out/tb.jsonl"; timeout -k 10 240 env "$@" >> "$out/tb.jsonl" 2>> "$out/tb.err" || exit $?; }
run TB_MIXED=1 TB_QBYTES=132 $tb $N 3 8:32768,16:131072,32:4096 8:32768,16:131072 16:131072,32:4096
run TB_MIXED=8 TB_QBYTES=132 $tb $N 3 1128:131072,32:4096 1128:131072 1128:131072,16:22528,32:4096
run TB_MIXED=4 TB_QBYTES=132 $tb $N 3 1064:131072,32:4096 1064:131072
run TB_MIXED=1 TB_QBYTES=0 $tb $N 3 8:32768,16:131072,32:4096 4:4096
exit 0
