#!/bin/bash
# Round-5 A/B batch 10 (repo root, GPU box): the refit block at 64 or 256
# lanes (build_rb64 / build_rb256: -DMW_REFIT_BLOCK) against 128, with the
# LDS sized for two thirds of the node capacity.
set -o pipefail
O=gpurun_out/ab15
mkdir -p $O
timeout -k 10 400 python tools/ab_bench.py --workload collisions --steps 20 --out $O/c \
    base rb64:LIB=build_rb64 rb256:LIB=build_rb256 base2 rb642:LIB=build_rb64 rb2562:LIB=build_rb256 \
    > $O/collisions.log 2>&1 || { tail -20 $O/collisions.log; exit 2; }
echo ab-done
