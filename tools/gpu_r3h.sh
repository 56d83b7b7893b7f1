set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
AEROGNN_LIB=aero-gnn_amd/aerognn/libaerognn_stamps.so timeout -k 10 200 python -u tools/edge_bwd_stamps.py > gpurun_out/r3h_stamps.log 2>&1 && \
timeout -k 10 200 python -u tools/debug_fused_edge.py > gpurun_out/r3h_dbg.log 2>&1 && \
AEROGNN_FUSED_EDGE_BWD=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > gpurun_out/r3h_bench.log 2>&1
