#!/bin/bash
# SQ issue / LDS counters of the narrowphase kernels on a workload (GPU box,
# repo root):  bash tools/sq_lds.sh <tag> [simple|collisions]
# Two PMC passes (8 SQ counters each), kernel-trace only, each under its own
# time limit; summary: python profiles/sq_summary.py gpurun_out/<tag> --out ...
set -euo pipefail
T=${1:-sqlds}
WL=${2:-simple}
OUT=$PWD/gpurun_out/$T
B="$PWD/bench.py --workload $WL --no-cpu-baseline --no-cpu-executor --no-roofline --ref-ticks 0 --settle 120 --steps 3 --warmup 1"
RX="narrowSATKernel|narrowContactKernel|solverKernel"
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex "$RX" --output-format csv -d $OUT/p1 -o run -- python3 $B > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAVES SQ_WAVE_CYCLES --kernel-include-regex "$RX" --output-format csv -d $OUT/p2 -o run -- python3 $B > $OUT/p2.log 2>&1
