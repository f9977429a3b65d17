#!/bin/bash
# Round-5 A/B batch 11 (repo root, GPU box): the export scan with each
# thread's counts held in registers (default) against the loop form
# (build_old): rocprofv3 kernel stats of one bench run each, then the GPU
# suite.
set -o pipefail
O=$PWD/gpurun_out/ab16
mkdir -p $O
R=$PWD
for v in new old; do
    if [ $v = old ]; then export MADRONA_MW_LIB=$R/gpu-ecs-madrona_amd/build_old/libmadrona_mw.so; fi
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $O/$v -o run -- python3 $R/bench.py --no-cpu-baseline --no-cpu-executor --ref-ticks 0 \
        --steps 20 --warmup 5 > $O/$v.log 2>&1) || exit 2
    grep -h "export" $(find $O/$v -name "*kernel_stats.csv") > $O/$v.export.txt
    find $O/$v -name "*kernel_trace.csv" -delete
done
unset MADRONA_MW_LIB
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 4; }
tail -1 $O/tests.log
echo ab-done
