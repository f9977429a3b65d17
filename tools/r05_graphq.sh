#!/bin/bash
# Round-5 experiment (repo root, GPU box): does the graph run the hull-plane
# branch beside SAT + contact?  bench.py under the HIP runtime's graph
# switches with the side stream on (MADRONA_MW_SIDE_STREAM=1), then a kernel
# trace with the side stream checked by
# tools/concurrency_check.py.
set -o pipefail
O=gpurun_out/gq
mkdir -p $O
timeout -k 10 400 python tools/ab_bench.py --workload collisions --steps 20 --out $O/c \
    base side:MADRONA_MW_SIDE_STREAM=1 sidenopc:MADRONA_MW_SIDE_STREAM=1,DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 \
    sideq8:MADRONA_MW_SIDE_STREAM=1,DEBUG_HIP_FORCE_GRAPH_QUEUES=8 base2 \
    > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 2; }
R=$PWD
(cd /tmp && export TMPDIR=/tmp && MADRONA_MW_SIDE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace \
    --output-format csv -d $R/$O/t -o run -- python3 $R/bench.py --no-cpu-baseline --no-cpu-executor \
    --ref-ticks 0 --steps 20 --warmup 5 > $R/$O/trace.log 2>&1) || exit 3
f=$(find $O/t -name "*kernel_trace.csv" | head -1)
python3 tools/concurrency_check.py $f > $O/plane.txt
rc=$?
find $O -name "*.csv" -delete
exit $rc
