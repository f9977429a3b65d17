set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo BENCHFAIL; tail -30 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
