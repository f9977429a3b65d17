#!/bin/bash
# Round-5 A/B batch (repo root, GPU box): findOverlaps occupancy variants and
# the re-verification of the pre-9e95308 flag-only dead ends.
# Variant builds it loads (built beforehand, in-tree, then removed):
#   make -C gpu-ecs-madrona_amd BUILD=build_ow5 EXTRA=-DMW_OVERLAP_WAVES=5 (ow6, ow8 likewise),
#   build_sol4/5 EXTRA=-DMW_SOLVER_WAVES_PER_EU=4/5, build_bits0 EXTRA=-DMW_SAT_BITS=0,
#   build_sat_split EXTRA=-DMW_SAT_SPLIT_STAGE=1, build_sat_g16 EXTRA=-DMW_SAT_GROUP=16,
#   build_sat_3w EXTRA=-DMW_SAT_MIN_BLOCKS=3.  Results: profiles/r05_ab_*.txt.
set -o pipefail
O=gpurun_out/ab2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sat_bits_gpu.py tests/test_collisions_gpu.py tests/test_overlap_dfs_gpu.py tests/test_simple_gpu.py tests/test_hulls_gpu.py tests/test_lds_fallback_gpu.py -x -q \
    --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 500 python tools/ab_bench.py --workload collisions --steps 20 --out $O/c \
    base ow5:LIB=build_ow5 ow6:LIB=build_ow6 ow8:LIB=build_ow8 sol4:LIB=build_sol4 sol5:LIB=build_sol5 \
    base2 ow8b:LIB=build_ow8 dfs0:MADRONA_MW_OVERLAP_DFS_LEAVES=0 > $O/collisions.log 2>&1 || { tail -20 $O/collisions.log; exit 2; }
timeout -k 10 500 python tools/ab_bench.py --workload simple --steps 50 --out $O/s \
    base bits0:LIB=build_bits0 split:LIB=build_sat_split g16:LIB=build_sat_g16 w3:LIB=build_sat_3w base2 bits0b:LIB=build_bits0 \
    > $O/simple.log 2>&1 || { tail -20 $O/simple.log; exit 3; }
echo ab-done
