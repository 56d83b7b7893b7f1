# Round-4 session k: the wgrad segment-sum tests (a fault ends the script), then an A/B of
# AEROGNN_WGRAD_SEG on the C3 train step, twice, alternating.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=${1:-r4k}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -v -k "segment_sums or wgrad or fused_edge" \
    --timeout 200 --timeout-method thread > gpurun_out/${T}_seg.log 2>&1
tail -2 gpurun_out/${T}_seg.log
B="bench.py --no-cpu-baseline --no-c4 --steps 12 --warmup 3"
for rep in 1 2; do
  for s in 0 1; do
    AEROGNN_WGRAD_SEG=$s timeout -k 10 300 python -u $B > gpurun_out/${T}_seg${s}_train${rep}.log 2>&1
  done
done
python tools/bench_summary.py gpurun_out/${T}_seg*_train*.log
