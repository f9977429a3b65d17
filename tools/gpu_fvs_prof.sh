#!/bin/bash
# Kernel trace of the fantasy_vs bench (run from the repo root on the GPU box):
#   bash tools/gpu_fvs_prof.sh TAG [extra bench_fvs args]
set -o pipefail
T=${1:-fvs}
shift || true
R=$PWD
mkdir -p gpurun_out/$T
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T/trace -o run -- python3 $R/tools/bench_fvs.py --no-cpu-baseline "$@" > $R/gpurun_out/$T/bench.log 2>&1 || { echo PROFFAIL; tail -20 $R/gpurun_out/$T/bench.log; exit 1; }
