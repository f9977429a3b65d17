#!/bin/bash
# Counters of the solver kernel cut after each phase (repo root, GPU box):
#   bash tools/solver_cut_pmc.sh <tag> [collisions|simple]
# needs the timing build:  make -C gpu-ecs-madrona_amd BUILD=build_cut EXTRA=-DMW_SAT_CUTS
# tools/sat_profile.py --solver-cuts relaunches the solver 20 times per cut on
# the last substep's inputs (cuts 1,2,3,4,5,6,0,7 in that order); one
# rocprofv3 --pmc pass per counter group, summarised by tools/solver_cut_summary.py.
set -o pipefail
T=$1; WL=${2:-collisions}
OUT=$PWD/gpurun_out/$T
R=$PWD
mkdir -p $OUT
export MADRONA_MW_LIB=$R/gpu-ecs-madrona_amd/build_cut/libmadrona_mw.so
timeout -k 10 200 python3 tools/sat_profile.py $WL --solver-cuts > $OUT/cuts.txt 2>&1 || { tail -5 $OUT/cuts.txt; exit 2; }
cat $OUT/cuts.txt
cd /tmp && export TMPDIR=/tmp
pass() {
    local name=$1; shift
    timeout -s KILL 200 rocprofv3 --pmc "$@" --kernel-include-regex solverKernel --output-format csv \
        -d $OUT/$name -o run -- python3 $R/tools/sat_profile.py $WL --solver-cuts > $OUT/$name.log 2>&1 \
        || { echo "pass $name failed rc=$?"; tail -5 $OUT/$name.log; }
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES
pass tatd TD_TD_BUSY_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum
find $OUT \( -name "*.db" -o -name "*kernel_trace.csv" \) -delete
cd $R && python3 tools/solver_cut_summary.py $OUT
