#!/bin/bash
# Round-5 A/B batch 3 (repo root, GPU box): solver register budget (2 waves /
# SIMD without spills vs 3 with) and the write-back batch.
set -o pipefail
O=gpurun_out/ab3
mkdir -p $O
timeout -k 10 500 python tools/ab_bench.py --workload collisions --steps 20 --out $O/c \
    base sol2:LIB=build_sol2 wb1:LIB=build_wb1 wb2:LIB=build_wb2 base2 sol2b:LIB=build_sol2 \
    > $O/collisions.log 2>&1 || { tail -20 $O/collisions.log; exit 2; }
timeout -k 10 500 python tools/ab_bench.py --workload simple --steps 50 --out $O/s \
    base sol2:LIB=build_sol2 wb1:LIB=build_wb1 base2 \
    > $O/simple.log 2>&1 || { tail -20 $O/simple.log; exit 3; }
echo ab-done
