#!/bin/bash
# One GPU iteration (repo root, GPU box): selected -m gpu tests, the
# fantasy_vs bench and the collisions bench, each under its own limit.
#   bash tools/gpu_iter.sh <outdir> ["pytest -k expr"]
set -o pipefail
O=gpurun_out/${1:-iter}
K=${2:-}
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" \
      > $O/tests.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
timeout -k 10 300 python -u tools/bench_fvs.py --no-cpu-baseline > $O/fvs.json 2> $O/fvs.err \
    || { echo FVSFAIL; tail -20 $O/fvs.err; exit 2; }
python3 -c "
import json; d = json.loads(open('$O/fvs.json').read().strip().splitlines()[-1]); r = d['roofline']
print('fvs', d['value'], d['ms_per_step'], r['ms_per_launch'], r['frac'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err \
    || { echo BENCHFAIL; tail -20 $O/bench.err; exit 3; }
python3 -c "
import json; d = json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r = d['roofline']
print('collisions', d['value'], d['ms_per_step'], r['kernel'], r['ms_per_launch'], r['frac'], d['reference_definition'])"
