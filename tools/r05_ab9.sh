#!/bin/bash
# Round-5 A/B batch 9 (repo root, GPU box): the refit kernel's LDS sized for
# two thirds of the node capacity with an in-place fallback per world
# (default) against the full capacity (build_old: HEAD before the change);
# then the whole GPU suite (with tests/test_refit_lds_cap_gpu.py).
set -o pipefail
O=gpurun_out/ab14
mkdir -p $O
timeout -k 10 300 python tools/ab_bench.py --workload collisions --steps 20 --out $O/c \
    base old:LIB=build_old base2 old2:LIB=build_old \
    > $O/collisions.log 2>&1 || { tail -20 $O/collisions.log; exit 2; }
timeout -k 10 250 python tools/ab_bench.py --workload simple --steps 50 --out $O/s \
    base old:LIB=build_old \
    > $O/simple.log 2>&1 || { tail -20 $O/simple.log; exit 3; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 4; }
tail -2 $O/tests.log
echo ab-done
