set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
AEROGNN_LIB=aero-gnn_amd/aerognn/libaerognn_stamps.so timeout -k 10 200 python -u tools/edge_bwd_stamps.py > gpurun_out/r3r_stamps.log 2>&1 && \
timeout -k 10 200 python -u tools/debug_fused_edge.py > gpurun_out/r3r_dbg.log 2>&1 && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fullsize.py -k fused > gpurun_out/r3r_fused_test.log 2>&1 && \
for L in libaerognn libaerognn_prev; do \
AEROGNN_LIB=aero-gnn_amd/aerognn/$L.so AEROGNN_FUSED_EDGE_BWD=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > gpurun_out/r3r_c3f_$L.log 2>&1 || exit 1; \
AEROGNN_LIB=aero-gnn_amd/aerognn/$L.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > gpurun_out/r3r_c3_$L.log 2>&1 || exit 1; \
done
