#!/bin/bash
# Round-5 A/B batch 7 (repo root, GPU box): the first substep's filter on the
# wave-per-world form (narrowFilterWaveKernel, default) against the
# block-per-world kernel (build_fb0: -DMW_FILTER_WAVE=0); then the whole GPU
# suite on the default build.
set -o pipefail
O=gpurun_out/ab12
mkdir -p $O
timeout -k 10 300 python tools/ab_bench.py --workload collisions --steps 20 --out $O/c \
    base fb0:LIB=build_fb0 base2 fb02:LIB=build_fb0 \
    > $O/collisions.log 2>&1 || { tail -20 $O/collisions.log; exit 2; }
timeout -k 10 250 python tools/ab_bench.py --workload simple --steps 50 --out $O/s \
    base fb0:LIB=build_fb0 \
    > $O/simple.log 2>&1 || { tail -20 $O/simple.log; exit 3; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 4; }
tail -2 $O/tests.log
echo ab-done
