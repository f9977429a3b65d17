#!/bin/bash
# Round profile collection on the GPU box (run from the repo root):
#   bash profiles/collect.sh rNN [workload] [steps] [warmup]   (collisions by default; simple)
# (a shorter window, e.g. 50 steps, keeps a slow workload's PMC passes short)
# kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate PMC passes
# (no sys/runtime trace with --pmc), each bounded by its own timeout; the
# bench's default window (steps 131-330), summarised over its 200 steps.
set -euo pipefail
R=${1:-r01}
WL=${2:-collisions}
STEPS=${3:-200}
WARM=${4:-10}
SETTLE=120
WIN="$((SETTLE + WARM + 1))-$((SETTLE + WARM + STEPS))"
OUT=$PWD/gpurun_out/prof_$R${2:+_$2}_w$WIN
B="$PWD/bench.py --no-cpu-baseline --no-cpu-executor --ref-ticks 0 --workload $WL --steps $STEPS --warmup $WARM"
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1
timeout -k 10 170 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "phys::" --output-format csv -d $OUT/fetch -o run -- python3 $B > $OUT/fetch.log 2>&1
timeout -k 10 170 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "phys::" --output-format csv -d $OUT/write -o run -- python3 $B > $OUT/write.log 2>&1
cd $OLDPWD
python3 profiles/pmc_traffic.py --trace $OUT/trace --fetch $OUT/fetch --write $OUT/write --steps $STEPS --timed-steps $WIN --out $OUT/traffic.json > /dev/null
python3 tools/prof_db.py $(find $OUT/trace -name "*.db" | head -1) $STEPS > $OUT/kernels.txt 2>/dev/null || true
