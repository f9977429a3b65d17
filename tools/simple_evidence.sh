#!/bin/bash
# configs[1] (simple_taskgraph) evidence over ONE window (GPU box, repo root):
#   bash tools/simple_evidence.sh rNN [steps]
# the bench line (steps 131..130+K), the kernel trace + PMC traffic of the
# same window (profiles/collect.sh), then the SQ issue / LDS counters of the
# narrowphase and solver kernels (tools/sq_lds.sh).  Each step time-limited.
set -o pipefail
R=${1:-r05}
K=${2:-50}
O=gpurun_out/${R}_simple
mkdir -p $O
timeout -k 10 400 python -u bench.py --workload simple --steps $K > $O/bench.json 2> $O/bench.err \
    || { echo BENCHFAIL; tail -20 $O/bench.err; exit 1; }
tail -c 300 $O/bench.json
timeout -k 10 900 bash profiles/collect.sh $R simple $K 10 || { echo COLLECTFAIL; exit 2; }
timeout -k 10 700 bash tools/sq_lds.sh ${R}_simple_sq simple || { echo SQFAIL; exit 3; }
python3 profiles/sq_summary.py gpurun_out/${R}_simple_sq --out gpurun_out/${R}_simple_sq/sq_summary.json > /dev/null || true
# the raw rocpd databases are summarised (kernels.txt); gpurun copies back at most 64 MiB
find gpurun_out -name "*.db" -delete
du -sh gpurun_out
echo done
