#!/bin/bash
# A/B the bench over library variants: bash tools/ab_bench.sh <tag> <build_dir>...
# (each variant: gpu-ecs-madrona_amd/<build_dir>/libmadrona_mw.so)
set -euo pipefail
T=$1; shift
mkdir -p gpurun_out/$T
for b in "$@"; do
  MADRONA_MW_LIB=$PWD/gpu-ecs-madrona_amd/$b/libmadrona_mw.so timeout -k 10 240 \
    python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/$T/$b.json 2> gpurun_out/$T/$b.err
done
