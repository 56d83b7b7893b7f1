# Round-4 session n: the float64-mode tests (new kernels; a crash ends the script), then the L2
# prefetch A/B of session m.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=${1:-r4n}
rc=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_f64.py -v -rP --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_f64.log 2>&1 || rc=$?
grep -E "passed|failed" gpurun_out/${T}_f64.log | tail -1
grep -E "::.*FAILED|Error" gpurun_out/${T}_f64.log | head -5 || true
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "f64 tests ended with status $rc"; exit $rc; fi
grep -q "Memory access fault\|Fatal Python error\|core dumped" gpurun_out/${T}_f64.log && exit 3
bash tools/gpu_r4m.sh ${T}
