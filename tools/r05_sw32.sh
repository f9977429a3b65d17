#!/bin/bash
# Two worlds per solver wave (MW_SOLVER_LANES=32): parity, then A/B.
# Variant build: make -C gpu-ecs-madrona_amd BUILD=build_sw32 EXTRA=-DMW_SOLVER_LANES=32
set -o pipefail
O=gpurun_out/sw32
mkdir -p $O
MADRONA_MW_LIB=$PWD/gpu-ecs-madrona_amd/build_sw32/libmadrona_mw.so timeout -k 10 400 python -u -m pytest \
    tests/test_collisions_gpu.py tests/test_simple_gpu.py tests/test_joints_gpu.py tests/test_lds_fallback_gpu.py \
    tests/test_hulls_gpu.py tests/test_sat_bits_gpu.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 \
    || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python tools/ab_bench.py --workload collisions --steps 20 --out $O/c \
    base sw32:LIB=build_sw32 base2 sw32b:LIB=build_sw32 > $O/c.log 2>&1 || exit 2
timeout -k 10 400 python tools/ab_bench.py --workload simple --steps 50 --out $O/s \
    base sw32:LIB=build_sw32 > $O/s.log 2>&1 || exit 3
echo sw32-done
