#!/bin/bash
# Round-end measurements on the GPU box (run from the repo root):
#   bash tools/gpu_final.sh TAG
# the GPU test suite, then the collisions bench (with both CPU legs), the
# simple bench, fantasy_vs (with its CPU leg) and the settled-window kernel
# profile; every step bounded by its own timeout, the first failure ends it.
set -o pipefail
T=${1:-final}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo BENCHFAIL; tail -30 $O/bench.log; exit 2; }
tail -1 $O/bench.log
timeout -k 10 300 python -u bench.py --workload simple > $O/simple.log 2>&1 || { echo SIMPLEFAIL; tail -30 $O/simple.log; exit 3; }
tail -1 $O/simple.log
timeout -k 10 400 python -u tools/bench_fvs.py > $O/fvs.log 2>&1 || { echo FVSFAIL; tail -30 $O/fvs.log; exit 4; }
tail -1 $O/fvs.log
bash tools/gpu_prof.sh $T/prof || exit 5
