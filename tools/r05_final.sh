#!/bin/bash
# Round-5 evidence on the GPU box (repo root):  bash tools/r05_final.sh <stage>...
#   tests    the whole -m gpu suite
#   bench    bench.py (collisions, configs[2], default window + CPU legs),
#            bench.py --workload simple --steps 50 (configs[1], steps 131-180:
#            the window the simple profiles cover), tools/bench_fvs.py (configs[4])
#   prof200  kernel trace + PMC traffic: collisions 131-330
#   prof     the same for collisions 126-145 and simple 131-180
#   fvsprof  kernel trace + stats of tools/bench_fvs.py's run (walk + resume kernels)
#   sq       SQ issue / LDS counters of the narrowphase and solver kernels (simple)
# Each step under its own time limit; stops at the first failure.
set -o pipefail
O=gpurun_out/r05
mkdir -p $O
# the raw traces are summarised on the box (traffic.json, kernels.txt,
# sq summaries); gpurun copies back at most 64 MiB
prune() {
    find gpurun_out \( -name "*.db" -o -name "*kernel_trace.csv" \) -delete
    find gpurun_out -path "*prof_r05*" -name "*counter_collection.csv" -delete
}
stop() { echo "FAILED: $1 (rc $2)"; prune; exit "$2"; }
for st in "$@"; do
    case $st in
    tests) bash tools/round_final.sh r05 tests || stop tests $? ;;
    bench)
        timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || stop bench $?
        timeout -k 10 500 python -u bench.py --workload simple --steps 50 > $O/simple_bench.json \
            2> $O/simple_bench.err || stop simple $?
        timeout -k 10 400 python -u tools/bench_fvs.py > $O/fvs_bench.json 2> $O/fvs_bench.err || stop fvs $?
        tail -c 200 $O/bench.json; tail -c 200 $O/simple_bench.json; tail -c 200 $O/fvs_bench.json ;;
    prof200)
        timeout -k 10 700 bash profiles/collect.sh r05 collisions 200 10 || stop prof_c200 $?
        prune ;;
    prof)
        timeout -k 10 400 bash profiles/collect.sh r05 collisions 20 5 || stop prof_c20 $?
        timeout -k 10 500 bash profiles/collect.sh r05 simple 50 10 || stop prof_s50 $?
        prune ;;
    fvsprof)
        R=$PWD
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
            -d $R/$O/fvsprof -o run -- python3 $R/tools/bench_fvs.py --no-cpu-baseline \
            > $R/$O/fvsprof.log 2>&1) || stop fvsprof $? ;;
    sq)
        timeout -k 10 700 bash tools/sq_lds.sh r05_simple_sq simple || stop sq $?
        python3 profiles/sq_summary.py gpurun_out/r05_simple_sq --out $O/simple_sq_summary.json > /dev/null
        prune ;;
    esac
done
prune
du -sh gpurun_out
echo final-done
