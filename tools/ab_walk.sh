#!/bin/bash
# World-walk A/B on the GPU box (repo root): fantasy_vs (configs[4]) under
# several variants, alternated round by round.
#   bash tools/ab_walk.sh <outdir> <rounds> name:WALK:LIBDIR[:FULLGRID] ...
# e.g. nodes:0:build walk:1:build walk8:1:build_w8 (LIBDIR under gpu-ecs-madrona_amd/)
set -o pipefail
OUT=${1:-gpurun_out/ab_walk}
N=${2:-2}
shift 2
mkdir -p $OUT
for i in $(seq 1 $N); do
  for v in "$@"; do
    IFS=: read name wk lib full <<< "$v"
    MADRONA_MW_LIB=gpu-ecs-madrona_amd/$lib/libmadrona_mw.so MADRONA_MW_WORLD_WALK=$wk MADRONA_MW_WALK_FULL_GRID=${full:-0} \
        timeout -k 10 300 python -u tools/bench_fvs.py --no-cpu-baseline ${BENCH_ARGS:-} \
        > $OUT/fvs_${name}_$i.json 2> $OUT/fvs_${name}_$i.err || { echo "FAILED $name rc $?"; exit 1; }
    python3 -c "
import json; d = json.loads(open('$OUT/fvs_${name}_$i.json').read().strip().splitlines()[-1])
print('$name', d['value'], d.get('ms_per_step'))"
  done
done
