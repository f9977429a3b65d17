#!/bin/bash
# Round-5 A/B batch 4 (repo root, GPU box): the SAT kernel's world sort on a
# block of its own (MW_SAT_SORT_ALONE=1, default) against block 0 sorting and
# then taking its share of the pairs (build_s0: -DMW_SAT_SORT_ALONE=0).
set -o pipefail
O=gpurun_out/ab4
mkdir -p $O
timeout -k 10 300 python tools/ab_bench.py --workload collisions --steps 20 --out $O/c \
    base s0:LIB=build_s0 base2 s02:LIB=build_s0 \
    > $O/collisions.log 2>&1 || { tail -20 $O/collisions.log; exit 2; }
timeout -k 10 250 python tools/ab_bench.py --workload simple --steps 50 --out $O/s \
    base s0:LIB=build_s0 base2 s02:LIB=build_s0 \
    > $O/simple.log 2>&1 || { tail -20 $O/simple.log; exit 3; }
echo ab-done
