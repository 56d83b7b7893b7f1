set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3w_smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r3w_bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --mode fwd --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3w_c3_fwd.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --mode fwd --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3w_c5_fwd.log 2>&1 && \
AEROGNN_FUSED_EDGE_BWD=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-c4 > gpurun_out/r3w_bench_split.log 2>&1
