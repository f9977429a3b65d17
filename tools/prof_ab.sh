#!/bin/bash
# rocprofv3 kernel stats of a short bench per library variant:
#   bash tools/prof_ab.sh <tag> <build_dir>...   (run on the GPU box)
set -o pipefail
export TMPDIR=/tmp
T=${1:-np1}; shift; mkdir -p gpurun_out/$T
for b in "$@"; do
  MADRONA_MW_LIB=$PWD/gpu-ecs-madrona_amd/$b/libmadrona_mw.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/$b -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 2 > gpurun_out/$T/$b.log 2>&1 || { echo FAIL $b; tail -20 gpurun_out/$T/$b.log; exit 1; }
  f=$(find gpurun_out/$T/$b -name '*kernel_stats.csv' | head -1)
  echo "== $b"; python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
for x in r:
  if any(k in x['Name'] for k in ('narrow','solver','Overlap','Plane','integrate')): print(x['Name'][:40], x['Calls'], x['AverageNs'])
"
done
