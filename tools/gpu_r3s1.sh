# Session r3s1: A/B of batched-load grouped-row kernels (seg_micro), then the kernel/op GPU tests
# on the new default build, then the C3 train bench line.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
timeout -k 10 240 python -u tools/seg_micro.py ab/libA_base.so ab/libB_s4_g2.so ab/libB_s8_g4.so ab/libB_s4_g8.so ab/libB_s16_g4.so aero-gnn_amd/aerognn/libaerognn.so > gpurun_out/r3s1_seg_micro.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_ops.py > gpurun_out/r3s1_tests.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 > gpurun_out/r3s1_bench.log 2>&1
