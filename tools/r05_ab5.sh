#!/bin/bash
# Round-5 A/B batch 5 (repo root, GPU box): the plane kernel with its hull
# tables read through LDS-typed pointers (narrowPlaneKernel, kGeo template)
# against the generic-pointer build (build_old: HEAD before the change), then
# the parity tests that cover the plane kernel and the forced-HBM variant.
# Re-run with O=ab9 for the SAT kernel's pose loads through global-typed
# pointers (loadPose) against HEAD, and with O=ab10 for the contact kernel
# with its hull tables staged into LDS after the clip buffers.
set -o pipefail
O=gpurun_out/ab10
mkdir -p $O
timeout -k 10 300 python tools/ab_bench.py --workload collisions --steps 20 --out $O/c \
    base old:LIB=build_old base2 old2:LIB=build_old \
    > $O/collisions.log 2>&1 || { tail -20 $O/collisions.log; exit 2; }
timeout -k 10 250 python tools/ab_bench.py --workload simple --steps 50 --out $O/s \
    base old:LIB=build_old \
    > $O/simple.log 2>&1 || { tail -20 $O/simple.log; exit 3; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_lds_fallback_gpu.py tests/test_collisions_gpu.py tests/test_sat_bits_gpu.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 4; }
tail -2 $O/tests.log
echo ab-done
