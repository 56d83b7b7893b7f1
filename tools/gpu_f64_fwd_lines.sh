# The float64 tests (with poolMGN), then the C3 and C5 forward-only lines.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=${1:-r4t}
rc=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_f64.py -v -rP --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_f64.log 2>&1 || rc=$?
grep -E "passed|failed" gpurun_out/${T}_f64.log | tail -1
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "f64 tests ended with status $rc"; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 --steps 10 --warmup 3 --mode fwd > gpurun_out/${T}_c3_fwd.log 2>&1
tail -1 gpurun_out/${T}_c3_fwd.log | cut -c1-200
timeout -k 10 500 python -u bench.py --no-cpu-baseline --no-c4 --config c5 --steps 5 --warmup 2 --mode fwd > gpurun_out/${T}_c5_fwd.log 2>&1
tail -1 gpurun_out/${T}_c5_fwd.log | cut -c1-200
