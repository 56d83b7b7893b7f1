# Session r3s4: node kernel receiver sums computed cooperatively into LDS (AGN_NODE_COOP=1, the
# new default build) against the per-lane walk (ab/libW_walk.so, AGN_NODE_COOP=0): bitwise tests,
# full-step bitwise check, C3 train and C5 forward A/B.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "aggregation_paths or resident or parity or golden or layer" > gpurun_out/r3s4_tests.log 2>&1
timeout -k 10 200 python -u tools/ab_outputs.py save gpurun_out/r3s4_a.pt > gpurun_out/r3s4_ab.log 2>&1
AEROGNN_LIB=ab/libW_walk.so timeout -k 10 200 python -u tools/ab_outputs.py save gpurun_out/r3s4_b.pt >> gpurun_out/r3s4_ab.log 2>&1
timeout -k 10 200 python -u tools/ab_outputs.py cmp gpurun_out/r3s4_a.pt gpurun_out/r3s4_b.pt >> gpurun_out/r3s4_ab.log 2>&1
rm -f gpurun_out/r3s4_a.pt gpurun_out/r3s4_b.pt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 > gpurun_out/r3s4_bench_coop.log 2>&1
AEROGNN_LIB=ab/libW_walk.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 > gpurun_out/r3s4_bench_walk.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --mode fwd --no-cpu-baseline --no-c4 > gpurun_out/r3s4_c5_coop.log 2>&1
AEROGNN_LIB=ab/libW_walk.so timeout -k 10 300 python -u bench.py --config c5 --mode fwd --no-cpu-baseline --no-c4 > gpurun_out/r3s4_c5_walk.log 2>&1
