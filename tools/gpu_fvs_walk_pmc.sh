#!/bin/bash
# fantasy_vs walk-unit evidence (repo root, GPU box): kernel trace + stats,
# then FETCH_SIZE and WRITE_SIZE in separate PMC passes, each bounded by its
# own limit; summarised by tools/fvs_walk_pmc.py.   bash tools/gpu_fvs_walk_pmc.sh TAG
set -o pipefail
T=${1:-fvs_walk}
R=$PWD
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/tools/bench_fvs.py --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $B > $O/trace.log 2>&1 || { echo TRACEFAIL; tail -20 $O/trace.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "worldWalkKernel|worldResumeKernel" --output-format csv -d $O/fetch -o run -- python3 $B > $O/fetch.log 2>&1 || { echo FETCHFAIL; tail -20 $O/fetch.log; exit 2; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "worldWalkKernel|worldResumeKernel" --output-format csv -d $O/write -o run -- python3 $B > $O/write.log 2>&1 || { echo WRITEFAIL; tail -20 $O/write.log; exit 3; }
cd $R
python3 tools/fvs_walk_pmc.py --trace $(find $O/trace -name "*kernel_trace.csv" | head -1) \
    --fetch $(find $O/fetch -name "*counter_collection.csv" | head -1) \
    --write $(find $O/write -name "*counter_collection.csv" | head -1) \
    --out $O/fvs_traffic.json || exit 4
cp $(find $O/trace -name "*kernel_stats.csv" | head -1) $O/fvs_kernel_stats.csv
tail -1 $O/trace.log | cut -c1-300
find $O \( -name "*.db" -o -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -size +20M -delete
