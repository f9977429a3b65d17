#!/bin/bash
# Counters of fantasy_vs with and without the world walk (experiment tool):
#   bash tools/walk_pmc.sh TAG      (repo root, GPU box)
# short bench_fvs runs (200 + 100 ticks), kernel trace + 3 PMC passes each.
set -o pipefail
T=${1:-walk_pmc}
R=$PWD
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/tools/bench_fvs.py --no-cpu-baseline --no-node-timing --preroll 200 --steps 100"
RX="FantasyVS|structuralCommit|worldWalk|worldResume"
for wk in 0 1; do
  export MADRONA_MW_WORLD_WALK=$wk
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/w$wk/trace -o run -- python3 $B > $O/w$wk.trace.log 2>&1 || { echo TRACEFAIL $wk; tail -5 $O/w$wk.trace.log; exit 1; }
  i=0
  for set in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $set --kernel-include-regex "$RX" --output-format csv -d $O/w$wk/p$i -o run -- python3 $B > $O/w$wk.p$i.log 2>&1 || { echo PMCFAIL $wk $i; tail -5 $O/w$wk.p$i.log; exit 2; }
  done
done
echo done
