set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > gpurun_out/r3k_c3.log 2>&1 && \
AEROGNN_LIB=aero-gnn_amd/aerognn/libaerognn_prev.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > gpurun_out/r3k_c3_prev.log 2>&1
