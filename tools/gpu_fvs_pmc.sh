#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the fantasy_vs tick kernels (separate passes):
#   bash tools/gpu_fvs_pmc.sh TAG
set -o pipefail
T=${1:-fvs_pmc}
R=$PWD
mkdir -p gpurun_out/$T
cd /tmp && export TMPDIR=/tmp
B="$R/tools/bench_fvs.py --no-cpu-baseline --worlds 16384 --preroll 600 --steps 100 --chunk 50"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "FantasyVS|structuralCommit" --output-format csv -d $R/gpurun_out/$T/fetch -o run -- python3 $B > $R/gpurun_out/$T/fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "FantasyVS|structuralCommit" --output-format csv -d $R/gpurun_out/$T/write -o run -- python3 $B > $R/gpurun_out/$T/write.log 2>&1 || exit 2
