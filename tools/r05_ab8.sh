#!/bin/bash
# Round-5 A/B batch 8 (repo root, GPU box): the solver compiled under the
# AMDGPU scheduler strategies (SOLVER_FLAGS="-fno-slp-vectorize -mllvm
# -amdgpu-sched-strategy=S", build_s_S; all at 3 waves per SIMD, 162-168
# VGPRs, no spills) against the default scheduler.
set -o pipefail
O=gpurun_out/ab13
mkdir -p $O
timeout -k 10 500 python tools/ab_bench.py --workload collisions --steps 20 --out $O/c \
    base ilp:LIB=build_s_max-ilp iilp:LIB=build_s_iterative-ilp minreg:LIB=build_s_iterative-minreg \
    base2 ilp2:LIB=build_s_max-ilp iilp2:LIB=build_s_iterative-ilp minreg2:LIB=build_s_iterative-minreg \
    > $O/collisions.log 2>&1 || { tail -20 $O/collisions.log; exit 2; }
timeout -k 10 300 python tools/ab_bench.py --workload simple --steps 50 --out $O/s \
    base ilp:LIB=build_s_max-ilp iilp:LIB=build_s_iterative-ilp minreg:LIB=build_s_iterative-minreg \
    > $O/simple.log 2>&1 || { tail -20 $O/simple.log; exit 3; }
echo ab-done
