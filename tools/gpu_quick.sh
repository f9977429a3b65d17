#!/bin/bash
# Quick GPU iteration (run from the repo root on the GPU box):
#   bash tools/gpu_quick.sh TAG [pytest -k expr]
# physics parity tests, then a short bench; each step under its own limit.
set -o pipefail
T=${1:-quick}
K=${2:-"collisions or joints or hulls or simple or lds"}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTFAIL; grep -E "Error|assert|FAIL" gpurun_out/${T}_tests.log | head -20; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-cpu-executor --steps 200 > gpurun_out/${T}_bench.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/${T}_bench.log; exit 1; }
grep '^{' gpurun_out/${T}_bench.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', d['value'], 'ms/step', d['ms_per_step'], 'dom', r['kernel'], r['ms_per_launch'], 'ms/launch', 'frac', r['frac'])"
