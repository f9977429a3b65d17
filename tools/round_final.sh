#!/bin/bash
# Round-end evidence on the GPU box (repo root):  bash tools/round_final.sh <rNN> <stage>...
#   tests    the whole -m gpu suite
#   bench    bench.py (collisions, configs[2]) and --workload simple (configs[1]),
#            both with the CPU baseline legs
#   fvs      tools/bench_fvs.py (configs[4])
#   fvsprof  fantasy_vs walk-unit trace + PMC traffic (tools/gpu_fvs_walk_pmc.sh)
#   sq       SQ / TA / TD / TCP counters of the solver and narrowphase kernels
#   prof     rocprofv3 kernel stats + PMC traffic over the bench windows
#            (collisions steps 131-330 and 126-145, simple 131-180)
# Each step under its own time limit; stops at the first fault / time limit.
set -o pipefail
R=${1:-r04}
shift
mkdir -p gpurun_out/$R
stop() { echo "FAILED: $1 (rc $2)"; exit "$2"; }
for st in "$@"; do
    case $st in
    tests)
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
            > gpurun_out/$R/tests.log 2>&1 || stop tests $?
        tail -2 gpurun_out/$R/tests.log ;;
    bench)
        timeout -k 10 400 python -u bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err \
            || stop bench $?
        timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/$R/bench20.json \
            2> gpurun_out/$R/bench20.err || stop bench20 $?
        timeout -k 10 400 python -u bench.py --workload simple --steps 50 > gpurun_out/$R/simple_bench.json \
            2> gpurun_out/$R/simple_bench.err || stop simple_bench $?
        for f in bench bench20 simple_bench; do
            python3 -c "
import json; d = json.loads(open('gpurun_out/$R/$f.json').read().strip().splitlines()[-1])
r = d['roofline']; c = d.get('cpu_baseline') or {}
print('$f', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('traffic'), c.get('value'))"
        done ;;
    fvs)
        timeout -k 10 400 python -u tools/bench_fvs.py > gpurun_out/$R/fvs_bench.json \
            2> gpurun_out/$R/fvs_bench.err || stop fvs $?
        tail -c 400 gpurun_out/$R/fvs_bench.json ;;
    fvsprof)
        timeout -k 10 1000 bash tools/gpu_fvs_walk_pmc.sh ${R}_fvs || stop fvsprof $? ;;
    sq)
        timeout -k 10 1000 bash tools/kernel_pmc.sh ${R}_sq "solverKernel|narrowPlaneKernel|narrowSATKernel|narrowContactKernel|findOverlaps" \
            || stop sq $?
        python3 profiles/sq_summary.py gpurun_out/${R}_sq --out gpurun_out/${R}_sq/sq.json || stop sq_summary $? ;;
    prof)
        timeout -k 10 700 bash profiles/collect.sh $R collisions 200 10 || stop prof_collisions $?
        timeout -k 10 400 bash profiles/collect.sh $R collisions 20 5 || stop prof_collisions20 $?
        timeout -k 10 500 bash profiles/collect.sh $R simple 50 10 || stop prof_simple $?
        ls gpurun_out | grep "prof_$R" ;;
    esac
done
