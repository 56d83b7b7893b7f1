set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T="python -u -m pytest -x -v --timeout 400 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_kernels.py -k "gathered or segment_sum2" > gpurun_out/r3f_kern.log 2>&1 && \
timeout -k 10 500 $T tests/test_gpu_dist.py -k rccl > gpurun_out/r3f_rccl.log 2>&1 && \
timeout -k 10 600 $T tests/test_gpu_fullsize.py -k "concat" > gpurun_out/r3f_concat.log 2>&1 && \
AEROGNN_LIB=aero-gnn_amd/aerognn/libaerognn_stamps.so timeout -k 10 200 python -u tools/edge_bwd_stamps.py > gpurun_out/r3f_stamps.log 2>&1 && \
timeout -k 10 200 python -u tools/debug_fused_edge.py > gpurun_out/r3f_dbg.log 2>&1 && \
AEROGNN_FUSED_EDGE_BWD=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > gpurun_out/r3f_bench.log 2>&1
