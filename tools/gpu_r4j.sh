# Round-4 session j: the new wgrad segment-sum test first (a fault ends the script), then the fused
# edge backward timing, the GPU suite parts that cover the backward, and an A/B of
# AEROGNN_WGRAD_SEG (dP_d from the dW_e pass) against the separate segment_sum launch.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=${1:-r4j}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -v -k "segment_sums or wgrad" --timeout 200 \
    --timeout-method thread > gpurun_out/${T}_seg.log 2>&1
tail -2 gpurun_out/${T}_seg.log
rc=0
timeout -k 10 200 python -u tools/edge_bwd_stamps.py > gpurun_out/${T}_ebtime.txt 2>&1 || rc=$?
head -2 gpurun_out/${T}_ebtime.txt | grep -v amdgpu || true
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "timing ended with status $rc"; exit $rc; fi
rc=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_bf16.py tests/test_gpu_kernels.py \
    tests/test_gpu_parity.py -v -rP --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || rc=$?
grep -E "passed|failed" gpurun_out/${T}_tests.log | tail -2
grep -E "::.*FAILED" gpurun_out/${T}_tests.log | head || true
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with status $rc"; exit $rc; fi
B="bench.py --no-cpu-baseline --no-c4 --steps 12 --warmup 3"
for rep in 1 2; do
  for s in 0 1; do
    AEROGNN_WGRAD_SEG=$s timeout -k 10 300 python -u $B > gpurun_out/${T}_seg${s}_train${rep}.log 2>&1
  done
done
python tools/bench_summary.py gpurun_out/${T}_seg*_train*.log
