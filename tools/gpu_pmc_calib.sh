#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration for 4-B and 16-B accesses (tests/diag/pmc_calib.hip)
set -o pipefail
R=$PWD
mkdir -p gpurun_out/calib
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/calib/fetch -o run -- $R/tests/diag/build/pmc_calib > $R/gpurun_out/calib/fetch.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/calib/write -o run -- $R/tests/diag/build/pmc_calib > $R/gpurun_out/calib/write.log 2>&1 || exit 2
