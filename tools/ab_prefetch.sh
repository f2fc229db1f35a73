set -e
run() { timeout -k 10 200 python3 tools/ab_old_new.py "$@" 2>&1 | grep " ms" | tail -1; }
run old quad c3 fused
run new quad c3 fused
run old quad c3 compact
run new quad c3 compact
