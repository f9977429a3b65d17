#!/bin/bash
# Texture-addresser / data / L1 counters for the physics kernels (run from
# the repo root on the GPU box): bash tools/mem_counters.sh <tag>
set -euo pipefail
T=${1:-mem}
OUT=$PWD/gpurun_out/$T
B="$PWD/bench.py --no-cpu-baseline --steps 3 --warmup 1"
RX="solverKernel|narrowSATKernel|narrowContactKernel|findOverlapsKernel|refitKernel|narrowFilterKernel|integrateKernel"
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE SQ_WAVES --kernel-include-regex "$RX" --output-format csv -d $OUT/p1 -o run -- python3 $B > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TA_FLAT_READ_WAVEFRONTS_sum TA_TOTAL_WAVEFRONTS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_RDRET_STALL_sum GRBM_GUI_ACTIVE SQ_WAVES --kernel-include-regex "$RX" --output-format csv -d $OUT/p2 -o run -- python3 $B > $OUT/p2.log 2>&1
