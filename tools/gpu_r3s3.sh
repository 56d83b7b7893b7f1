# Session r3s3: receiver aggregation fused into the resident edge kernel (AEROGNN_EDGE_AGG, on by
# default) against the node kernel's walk: bitwise test, C3 train and C5 forward A/B, full-step
# bitwise check.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "aggregation_paths or fused_edge_bwd or resident" > gpurun_out/r3s3_tests.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 > gpurun_out/r3s3_bench_fused.log 2>&1
AEROGNN_EDGE_AGG=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 > gpurun_out/r3s3_bench_walk.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --mode fwd --no-cpu-baseline --no-c4 > gpurun_out/r3s3_c5_fused.log 2>&1
AEROGNN_EDGE_AGG=0 timeout -k 10 300 python -u bench.py --config c5 --mode fwd --no-cpu-baseline --no-c4 > gpurun_out/r3s3_c5_walk.log 2>&1
timeout -k 10 200 python -u tools/ab_outputs.py save gpurun_out/r3s3_a.pt > gpurun_out/r3s3_ab.log 2>&1
AEROGNN_EDGE_AGG=0 timeout -k 10 200 python -u tools/ab_outputs.py save gpurun_out/r3s3_b.pt >> gpurun_out/r3s3_ab.log 2>&1
timeout -k 10 200 python -u tools/ab_outputs.py cmp gpurun_out/r3s3_a.pt gpurun_out/r3s3_b.pt >> gpurun_out/r3s3_ab.log 2>&1
rm -f gpurun_out/r3s3_a.pt gpurun_out/r3s3_b.pt
