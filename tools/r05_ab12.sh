#!/bin/bash
# Round-5 A/B batch 12 (repo root, GPU box): the refit LDS capacity at 103
# and 98 nodes (13 / 14 blocks per CU; worlds past it refit in place)
# against the default two thirds of 172 (115 nodes, 12 blocks per CU).
set -o pipefail
O=gpurun_out/ab17
mkdir -p $O
timeout -k 10 400 python tools/ab_bench.py --workload collisions --steps 20 --out $O/c \
    base n103:MADRONA_MW_REFIT_LDS_NODES=103 n98:MADRONA_MW_REFIT_LDS_NODES=98 base2 \
    n1032:MADRONA_MW_REFIT_LDS_NODES=103 n982:MADRONA_MW_REFIT_LDS_NODES=98 \
    > $O/collisions.log 2>&1 || { tail -20 $O/collisions.log; exit 2; }
echo ab-done
