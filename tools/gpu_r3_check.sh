#!/bin/bash
# Round-3 check on the GPU box: collisions parity, then the bench kernel
# profile (settled window), refit / findOverlaps PMC traffic and the
# fantasy_vs kernel trace.  bash tools/gpu_r3_check.sh TAG
set -o pipefail
T=${1:-r3}
R=$PWD
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_collisions_gpu.py tests/test_joints_gpu.py tests/test_hulls_gpu.py tests/test_lds_fallback_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
bash tools/gpu_prof.sh $T/prof || exit 2
bash tools/gpu_refit_pmc.sh || exit 3
