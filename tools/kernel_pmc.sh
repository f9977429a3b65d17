#!/bin/bash
# Memory-pipeline / issue counters for chosen kernels (repo root, GPU box):
#   bash tools/kernel_pmc.sh <tag> <kernel regex> [bench args...]
# One rocprofv3 --pmc pass per counter group (within the per-block limits:
# 8 SQ, 4 TCP, 2 TA, 2 TD, 4 TCC, 2 GRBM), kernel trace only, each pass
# under its own kill timer; the counter list of the box goes to counters.txt.
set -o pipefail
T=$1; RX=$2; shift 2
OUT=$PWD/gpurun_out/$T
B="$PWD/bench.py --no-cpu-baseline --steps 3 --warmup 1 $*"
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
pass() {
    local name=$1; shift
    timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$RX" --output-format csv \
        -d $OUT/$name -o run -- python3 $B > $OUT/$name.log 2>&1 || { echo "pass $name failed rc=$?"; tail -5 $OUT/$name.log; }
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS
pass sq2 SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES
pass ta TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT
pass td TD_TD_BUSY_sum TD_SPI_STALL_sum
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum
pass ic SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVES
find $OUT \( -name "*.db" -o -name "*kernel_trace.csv" \) -delete
echo pmc-done
