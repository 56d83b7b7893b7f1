# Round-4 session b: A/B of the current build (B) against build_ab/libA.so (A): bitwise outputs of a
# full C3 bf16 step + an fp32 step, then the C3 train line of each (alternating), the VALU
# issue-cost micro-benchmark, and the fused / split / aggregation GPU tests on B.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=${1:-r4b}
timeout -k 10 300 ./tools/micro/valu_cost > gpurun_out/${T}_valu_cost.txt 2>&1
cat gpurun_out/${T}_valu_cost.txt
AEROGNN_LIB=build_ab/libA.so timeout -k 10 300 python -u tools/ab_outputs.py save gpurun_out/${T}_A.pt > gpurun_out/${T}_ab.txt 2>&1
timeout -k 10 300 python -u tools/ab_outputs.py save gpurun_out/${T}_B.pt >> gpurun_out/${T}_ab.txt 2>&1
python tools/ab_outputs.py cmp gpurun_out/${T}_A.pt gpurun_out/${T}_B.pt >> gpurun_out/${T}_ab.txt 2>&1 || true
rm -f gpurun_out/${T}_A.pt gpurun_out/${T}_B.pt
tail -25 gpurun_out/${T}_ab.txt
B="bench.py --no-cpu-baseline --no-c4 --steps 15 --warmup 3"
AEROGNN_LIB=build_ab/libA.so timeout -k 10 300 python -u $B > gpurun_out/${T}_bench_A1.log 2>&1
timeout -k 10 300 python -u $B > gpurun_out/${T}_bench_B1.log 2>&1
AEROGNN_LIB=build_ab/libA.so timeout -k 10 300 python -u $B > gpurun_out/${T}_bench_A2.log 2>&1
timeout -k 10 300 python -u $B > gpurun_out/${T}_bench_B2.log 2>&1
python tools/bench_summary.py gpurun_out/${T}_bench_*.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_bf16.py tests/test_gpu_kernels.py -v -rP \
    --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || true
grep -E "passed|failed" gpurun_out/${T}_tests.log | tail -3
