#!/bin/bash
# Round-5 A/B batch 3 (repo root, GPU box): register budgets -- the solver
# (2 waves / SIMD without spills vs 3 with), its write-back batch, and the
# narrowphase kernels pinned to more waves per SIMD.
# Variant builds: build_sol2 (-DMW_SOLVER_WAVES_PER_EU=2), build_wb1/2
#   (-DMW_SOLVER_WRITE_BATCH=1/2), build_flt8 (-DMW_FILTER_WAVES=8), build_pl5/6
#   (-DMW_PLANE_WAVES), build_ct5/6 (-DMW_CONTACT_WAVES), build_int8
#   (-DMW_INTEGRATE_WAVES=8).  Results: profiles/r05_ab_occupancy.txt.
set -o pipefail
O=gpurun_out/ab3
mkdir -p $O
timeout -k 10 900 python tools/ab_bench.py --workload collisions --steps 20 --out $O/c \
    base sol2:LIB=build_sol2 wb1:LIB=build_wb1 wb2:LIB=build_wb2 flt8:LIB=build_flt8 pl5:LIB=build_pl5 \
    pl6:LIB=build_pl6 ct5:LIB=build_ct5 ct6:LIB=build_ct6 int8:LIB=build_int8 base2 \
    > $O/collisions.log 2>&1 || { tail -20 $O/collisions.log; exit 2; }
timeout -k 10 250 python tools/ab_bench.py --workload simple --steps 50 --out $O/s \
    base sol2:LIB=build_sol2 base2 \
    > $O/simple.log 2>&1 || { tail -20 $O/simple.log; exit 3; }
echo ab-done
