#!/bin/bash
# GPU iteration loop (run from the repo root on the GPU box):
#   bash tools/gpu_check.sh [pytest -k expr]
# physics parity tests, a short bench and (with the profiling build) the
# solver phase split, each under its own timeout; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
K=${1:-"collisions or joints or simple or hulls"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/check_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/check_tests.log; exit 1; }
tail -2 gpurun_out/check_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 100 > gpurun_out/check_bench.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/check_bench.log; exit 1; }
tail -1 gpurun_out/check_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms/step', d['ms_per_step'], {k: v['ms_per_launch'] for k, v in d['nodes'].items()})"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 100 > gpurun_out/check_bench_nr.log 2>&1 || { echo BENCHFAIL2; tail -20 gpurun_out/check_bench_nr.log; exit 1; }
tail -1 gpurun_out/check_bench_nr.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('no-roofline value', d['value'], 'ms/step', d['ms_per_step'])"
if [ -f gpu-ecs-madrona_amd/build_prof/libmadrona_mw.so ]; then
  MADRONA_MW_LIB=gpu-ecs-madrona_amd/build_prof/libmadrona_mw.so timeout -k 10 200 python tools/solver_profile.py
fi
