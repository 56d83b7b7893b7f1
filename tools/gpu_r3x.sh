set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
timeout -k 10 600 python -u bench.py > gpurun_out/r3x_bench.log 2>&1
