#!/bin/bash
# SAT round on the GPU box: parity tests on the current build (and on the
# builds named in $TEST_LIBS), bench.py A/B over $VARIANTS (tools/ab_bench.py
# syntax) on configs[1], then the phase-cut timing build on both workloads.
# Stops at the first fault / time limit.
mkdir -p gpurun_out
T=${1:-r4_sat}
VARIANTS=${VARIANTS:-"new old:LIB=build_ab"}
TESTS="tests/test_collisions_gpu.py tests/test_simple_gpu.py tests/test_hulls_gpu.py tests/test_lds_fallback_gpu.py"
for lib in build ${TEST_LIBS}; do
    MADRONA_MW_LIB=gpu-ecs-madrona_amd/$lib/libmadrona_mw.so timeout -k 10 400 python -u -m pytest -x -q \
        --timeout 200 --timeout-method thread $TESTS > gpurun_out/${T}_tests_$lib.log 2>&1
    rc=$?
    echo "tests [$lib] rc=$rc"; tail -2 gpurun_out/${T}_tests_$lib.log
    if [ $rc -gt 1 ]; then exit $rc; fi
done
python -u tools/ab_bench.py --workload simple --out gpurun_out/${T} $VARIANTS || exit $?
for cut in ${CUT_LIBS:-build_cut}; do
    [ -f gpu-ecs-madrona_amd/$cut/libmadrona_mw.so ] || continue
    for wl in simple collisions; do
        echo "== $cut $wl"
        MADRONA_MW_LIB=gpu-ecs-madrona_amd/$cut/libmadrona_mw.so timeout -k 10 120 \
            python -u tools/sat_profile.py $wl --cuts > gpurun_out/${T}_${cut}_$wl.txt 2>&1
        rc=$?
        grep -v amdgpu.ids gpurun_out/${T}_${cut}_$wl.txt
        [ $rc -eq 0 ] || exit $rc
    done
done
