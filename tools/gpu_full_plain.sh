#!/bin/bash
# Full GPU check + the PLAIN PMC passes + the default bench (GPU box).
set -o pipefail
bash tools/gpu_full.sh || exit $?
bash tools/prof_r2.sh plain || exit $?
ls gpurun_out/prof/
