#!/bin/bash
# Round-5 A/B batch 6 (repo root, GPU box): the plane kernel without its
# software pipeline (build_pp0: -DMW_PLANE_PIPE=0, 118 VGPRs) and pinned to 5
# or 6 waves per SIMD (build_pp0w5 / build_pp0w6, -DMW_PLANE_WAVES).
set -o pipefail
O=gpurun_out/ab11
mkdir -p $O
timeout -k 10 400 python tools/ab_bench.py --workload collisions --steps 20 --out $O/c \
    base pp0:LIB=build_pp0 pp0w5:LIB=build_pp0w5 pp0w6:LIB=build_pp0w6 base2 pp02:LIB=build_pp0 \
    pp0w52:LIB=build_pp0w5 pp0w62:LIB=build_pp0w6 \
    > $O/collisions.log 2>&1 || { tail -20 $O/collisions.log; exit 2; }
echo ab-done
