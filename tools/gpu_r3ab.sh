set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
timeout -k 10 300 python -u tools/wgrad_micro.py > gpurun_out/r3ab_wgrad_micro.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "wgrad or mlp or concat or encoder or bsms" > gpurun_out/r3ab_tests.log 2>&1 && \
for rep in 1 2; do timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > gpurun_out/r3ab_bench_$rep.log 2>&1 || exit 1; done
