#!/bin/bash
# A/B driver (repo root, GPU box):  bash tools/ab_run.sh <out> <workload> <steps> [-k tests] variant...
#   each variant LABEL[:VAR=VAL,...] as tools/ab_bench.py takes them (LIB=<build dir>);
#   with -k EXPR the -m gpu tests matching EXPR run first (default library).
# Each step under its own time limit; stops at the first failure.
set -o pipefail
O=gpurun_out/$1; W=$2; S=$3; shift 3
mkdir -p $O
if [ "$1" = "-k" ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$2" \
        > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
    tail -1 $O/tests.log
    shift 2
fi
timeout -k 10 900 python tools/ab_bench.py --workload $W --steps $S --out $O/ab "$@" > $O/ab.log 2>&1 \
    || { tail -20 $O/ab.log; exit 3; }
cat $O/ab.log
