#!/bin/bash
# Steps-per-graph A/B (repo root, GPU box): parity with K = 8, then
# fantasy_vs and collisions at K = 1 / 8 / 16, alternated.
set -o pipefail
O=gpurun_out/spg
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fvs_gpu.py tests/test_world_walk_gpu.py \
    tests/test_collisions_gpu.py tests/test_multi_step_graph_gpu.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 \
    || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for K in 1 16; do
    MADRONA_MW_STEPS_PER_GRAPH=$K timeout -k 10 200 python -u tools/bench_fvs.py --no-cpu-baseline \
        > $O/fvs_k${K}_$r.json 2> $O/fvs_k${K}_$r.err || exit 2
    python3 -c "import json; d=json.loads(open('$O/fvs_k${K}_$r.json').read().strip().splitlines()[-1]); print('fvs K=$K', d['value'], d['ms_per_step'])"
  done
done
for K in 1 16; do
  MADRONA_MW_STEPS_PER_GRAPH=$K timeout -k 10 200 python -u tools/bench_fvs.py --no-cpu-baseline --no-node-timing \
      > $O/fvsu_k$K.json 2> $O/fvsu_k$K.err || exit 4
  python3 -c "import json; d=json.loads(open('$O/fvsu_k$K.json').read().strip().splitlines()[-1]); print('fvs untimed K=$K', d['value'], d['ms_per_step'])"
done
for K in 1 16; do
  MADRONA_MW_STEPS_PER_GRAPH=$K timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-cpu-executor --ref-ticks 0 \
      --steps 20 --warmup 5 > $O/c_k$K.json 2> $O/c_k$K.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/c_k$K.json').read().strip().splitlines()[-1]); print('collisions K=$K', d['value'], d['ms_per_step'])"
done
echo spg-done
