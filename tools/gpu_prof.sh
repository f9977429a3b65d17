#!/bin/bash
# Kernel-time profile of the bench's settled window (run from the repo root
# on the GPU box):  bash tools/gpu_prof.sh TAG [extra bench args]
# rocprofv3 kernel trace of a default bench run, summarised per kernel over
# its 200 timed steps by tools/prof_db.py.
set -o pipefail
T=${1:-prof}
shift || true
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/$T -o run -- python3 $R/bench.py --no-cpu-baseline --no-cpu-executor "$@" > $R/gpurun_out/${T}_bench.log 2>&1 || { echo PROFFAIL; tail -20 $R/gpurun_out/${T}_bench.log; exit 1; }
cd $R
python3 tools/prof_db.py $(find gpurun_out/$T -name "*.db" | head -1) 200 | tee gpurun_out/${T}_kernels.txt
grep '^{' gpurun_out/${T}_bench.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms/step', d['ms_per_step'])"
