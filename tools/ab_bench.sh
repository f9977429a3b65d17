#!/bin/bash
# A/B the bench over library variants: bash tools/ab_bench.sh <tag> <build_dir>...
# (each variant: gpu-ecs-madrona_amd/<build_dir>/libmadrona_mw.so); two
# rounds in alternating order; prints ms/step and the per-node launch times.
set -euo pipefail
T=$1; shift
mkdir -p gpurun_out/$T
for round in 1 2; do
  for b in "$@"; do
    MADRONA_MW_LIB=$PWD/gpu-ecs-madrona_amd/$b/libmadrona_mw.so timeout -k 10 240 \
      python bench.py --no-cpu-baseline --steps 100 --warmup 5 > gpurun_out/$T/$b.$round.json 2> gpurun_out/$T/$b.$round.err
    tail -1 gpurun_out/$T/$b.$round.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$b', $round, 'ms/step', d['ms_per_step'], {k[:6]: v['ms_per_launch'] for k, v in d['nodes'].items()}, 'dom', d['roofline']['kernel'], d['roofline']['ms_per_launch'])"
  done
done
