#!/bin/bash
# SQ counters of the collisions physics kernels (GPU box, repo root).
set -o pipefail
T=r05_coll_sq
sed 's/^RX=.*/RX="narrowPlaneKernel|narrowFilterKernel|solverKernel|narrowContactKernel|refitKernel|findOverlapsSmallKernel|narrowSATKernel"/' tools/sq_lds.sh > /tmp/sq_coll.sh
timeout -k 10 700 bash /tmp/sq_coll.sh $T collisions || exit 1
python3 profiles/sq_summary.py gpurun_out/$T --out gpurun_out/$T/sq_summary.json
echo sq-done
