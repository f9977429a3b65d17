#!/bin/bash
# Round-5 GPU batch (repo root): full -m gpu suite, configs[1] evidence over
# one window, solver worlds-per-block A/B.  Stops at the first failure.
set -o pipefail
bash tools/round_final.sh r05 tests || exit 1
bash tools/simple_evidence.sh r05 50 || exit 2
timeout -k 10 900 python tools/ab_bench.py --workload simple --steps 50 --out gpurun_out/ab_sw \
    sw1 sw2:LIB=build_sw2 sw4:LIB=build_sw4 sw1b sw4b:LIB=build_sw4 || exit 3
timeout -k 10 600 python tools/ab_bench.py --workload collisions --steps 50 --out gpurun_out/ab_sw \
    sw1 sw2:LIB=build_sw2 sw4:LIB=build_sw4 || exit 4
echo batch-done
