set -o pipefail
R=$PWD; mkdir -p gpurun_out/refit
timeout -k 10 200 python -u -m pytest tests/test_collisions_gpu.py tests/test_lds_fallback_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/refit/tests.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-cpu-executor --steps 10 --warmup 2"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "refit|findOverlaps" --output-format csv -d $R/gpurun_out/refit/fetch -o run -- python3 $B > $R/gpurun_out/refit/fetch.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "refit|findOverlaps" --output-format csv -d $R/gpurun_out/refit/write -o run -- python3 $B > $R/gpurun_out/refit/write.log 2>&1 || exit 3
