#!/bin/bash
# SQ counters for the physics kernels (run from the repo root on the GPU box):
#   bash tools/sq_counters.sh <tag>
# Two PMC passes (8 SQ slots each), kernel-trace only, each under its own timeout.
set -euo pipefail
T=${1:-sq}
OUT=$PWD/gpurun_out/$T
B="$PWD/bench.py --no-cpu-baseline --steps 3 --warmup 1"
RX="solverKernel|narrowSATKernel|narrowContactKernel|narrowPlaneKernel|findOverlapsKernel|refitKernel|narrowFilterKernel|integrateKernel|bvhRebuildWaveKernel|leafUpdateKernel"
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex "$RX" --output-format csv -d $OUT/p1 -o run -- python3 $B > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM --kernel-include-regex "$RX" --output-format csv -d $OUT/p2 -o run -- python3 $B > $OUT/p2.log 2>&1
# instruction-cache pass (large kernels: solver / narrowphase)
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQC_ICACHE_MISSES_DUPLICATE --kernel-include-regex "$RX" --output-format csv -d $OUT/p3 -o run -- python3 $B > $OUT/p3.log 2>&1
