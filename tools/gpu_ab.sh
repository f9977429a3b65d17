#!/bin/bash
# A/B of one environment switch on the collisions bench (run from the repo
# root on the GPU box):  bash tools/gpu_ab.sh TAG VAR [bench args]
# runs bench.py with VAR=0 and with VAR unset, twice each, interleaved.
set -o pipefail
T=${1:-ab}
V=$2
shift 2
O=gpurun_out/$T
mkdir -p $O
for i in 1 2; do
  env $V=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-cpu-executor "$@" > $O/off$i.log 2>&1 || { echo OFFFAIL; tail -20 $O/off$i.log; exit 1; }
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-cpu-executor "$@" > $O/on$i.log 2>&1 || { echo ONFAIL; tail -20 $O/on$i.log; exit 2; }
  for k in off on; do
    grep '^{' $O/$k$i.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline'] or {}; print('$k$i', d['value'], d['ms_per_step'], {n: v['ms_per_launch'] for n, v in d['nodes'].items()})"
  done
done
