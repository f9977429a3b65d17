#!/bin/bash
# A/B of the SAT kernel: parity tests on the current build, then bench.py
# --workload simple on the current build and on build_ab (HEAD), and the
# collisions bench on the current build.  Stops at any fault / timeout.
mkdir -p gpurun_out
T=${1:-r4_sat}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_collisions_gpu.py tests/test_simple_gpu.py tests/test_hulls_gpu.py \
    tests/test_lds_fallback_gpu.py > gpurun_out/${T}_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/${T}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u bench.py --workload simple --no-cpu-baseline --no-cpu-executor \
    > gpurun_out/${T}_simple_new.json 2>gpurun_out/${T}_err.log || exit $?
MADRONA_MW_LIB=gpu-ecs-madrona_amd/build_ab/libmadrona_mw.so timeout -k 10 200 python -u bench.py \
    --workload simple --no-cpu-baseline --no-cpu-executor > gpurun_out/${T}_simple_old.json \
    2>>gpurun_out/${T}_err.log || exit $?
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cpu-executor \
    > gpurun_out/${T}_coll_new.json 2>>gpurun_out/${T}_err.log || exit $?
for f in gpurun_out/${T}_*.json; do
    python -c "
import json; d = json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', d['value'], {k: v['ms_per_launch'] for k, v in d['nodes'].items()})"
done
