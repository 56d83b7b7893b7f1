set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=${1:-r4g}
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_bf16.py tests/test_gpu_kernels.py tests/test_gpu_parity.py -v -rP \
    --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || true
grep -E "passed|failed" gpurun_out/${T}_tests.log | tail -2
grep -E "::.*FAILED" gpurun_out/${T}_tests.log | head || true
bash tools/gpu_ab.sh $T build_ab/libP.so
