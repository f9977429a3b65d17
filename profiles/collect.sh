#!/bin/bash
# Round profile collection on the GPU box (run from the repo root):
#   bash profiles/collect.sh rNN
# kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate PMC passes
# (no sys/runtime trace with --pmc), each bounded by its own timeout.
set -euo pipefail
R=${1:-r01}
OUT=$PWD/gpurun_out/prof_$R
B="$PWD/bench.py --no-cpu-baseline --no-cpu-executor --steps 10 --warmup 2"
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "phys::" --output-format csv -d $OUT/fetch -o run -- python3 $B > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "phys::" --output-format csv -d $OUT/write -o run -- python3 $B > $OUT/write.log 2>&1
