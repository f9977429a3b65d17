#!/bin/bash
# Kernel trace of tools/bench_fvs.py with its live node timing (experiment
# tool): per-kernel durations of the walk in timed vs untimed ticks.
set -o pipefail
O=$PWD/gpurun_out/${1:-walk_trace}
mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/tools/bench_fvs.py --no-cpu-baseline ${TRACE_ARGS:---preroll 200 --steps 100} > $O/trace.log 2>&1 || { echo TRACEFAIL; tail -5 $O/trace.log; exit 1; }
echo done
