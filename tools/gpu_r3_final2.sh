#!/bin/bash
# Round-3 closing lines on the GPU box: the three bench lines (each with its
# CPU legs) and the simple workload's PMC traffic over a 50-step window.
set -o pipefail
O=gpurun_out/r3f2
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo BENCHFAIL; tail -30 $O/bench.log; exit 2; }
tail -1 $O/bench.log
timeout -k 10 300 python -u bench.py --workload simple > $O/simple.log 2>&1 || { echo SIMPLEFAIL; tail -30 $O/simple.log; exit 3; }
tail -1 $O/simple.log
timeout -k 10 400 python -u tools/bench_fvs.py > $O/fvs.log 2>&1 || { echo FVSFAIL; tail -30 $O/fvs.log; exit 4; }
tail -1 $O/fvs.log
bash profiles/collect.sh r03 simple 50 || { echo PMCFAIL; exit 5; }
cat gpurun_out/prof_r03_simple/traffic.json | head -c 3000
