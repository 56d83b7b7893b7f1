set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
for L in libaerognn libaerognn_var libaerognn libaerognn_var; do \
AEROGNN_LIB=aero-gnn_amd/aerognn/$L.so AEROGNN_FUSED_EDGE_BWD=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > gpurun_out/r3s_c3f_$L.log 2>&1 || exit 1; \
done
