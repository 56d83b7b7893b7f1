set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
timeout -k 10 200 python -u tools/debug_fused_edge.py > gpurun_out/r3_dbg.log 2>&1 && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fullsize.py > gpurun_out/r3a_fullsize.log 2>&1 ; \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > gpurun_out/r3a_bench.log 2>&1 && \
AEROGNN_FUSED_EDGE_BWD=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > gpurun_out/r3a_bench_split.log 2>&1
