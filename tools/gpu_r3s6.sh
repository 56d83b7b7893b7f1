# Session r3s6: node kernel receiver sums computed walked first with two member rows in flight (AGN_WALK2=1, the
# new default build) against the per-lane walk (ab/libW_walk.so, AGN_WALK2=0): bitwise tests,
# full-step bitwise check, C3 train and C5 forward A/B.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "aggregation_paths or resident or parity or golden or layer" > gpurun_out/r3s6_tests.log 2>&1
timeout -k 10 200 python -u tools/ab_outputs.py save gpurun_out/r3s6_a.pt > gpurun_out/r3s6_ab.log 2>&1
AEROGNN_LIB=ab/libW_walk.so timeout -k 10 200 python -u tools/ab_outputs.py save gpurun_out/r3s6_b.pt >> gpurun_out/r3s6_ab.log 2>&1
timeout -k 10 200 python -u tools/ab_outputs.py cmp gpurun_out/r3s6_a.pt gpurun_out/r3s6_b.pt >> gpurun_out/r3s6_ab.log 2>&1
rm -f gpurun_out/r3s6_a.pt gpurun_out/r3s6_b.pt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 > gpurun_out/r3s6_bench_w2.log 2>&1
AEROGNN_LIB=ab/libW_walk.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 > gpurun_out/r3s6_bench_walk.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --mode fwd --no-cpu-baseline --no-c4 > gpurun_out/r3s6_c5_w2.log 2>&1
AEROGNN_LIB=ab/libW_walk.so timeout -k 10 300 python -u bench.py --config c5 --mode fwd --no-cpu-baseline --no-c4 > gpurun_out/r3s6_c5_walk.log 2>&1
