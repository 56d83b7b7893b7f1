# Round-end closing set on one box: the GPU suite, the smoke check and the default bench line
# (tools/gpu_suite_bench.sh), then the forward-only C3 and C5 lines. Each step has its own limit;
# the script stops at the first failure of a bench step.
set -e
set -o pipefail
T=${1:-r6z}
bash tools/gpu_suite_bench.sh $T
export AEROGNN_MEMLOG=0
timeout -k 10 300 python -u bench.py --mode fwd --steps 20 --warmup 5 --no-cpu-baseline --no-c4 > gpurun_out/${T}_bench_c3_fwd.log 2>&1
tail -1 gpurun_out/${T}_bench_c3_fwd.log | cut -c1-200
timeout -k 10 400 python -u bench.py --config c5 --mode fwd --steps 10 --warmup 3 --no-cpu-baseline --no-c4 > gpurun_out/${T}_bench_c5_fwd.log 2>&1
tail -1 gpurun_out/${T}_bench_c5_fwd.log | cut -c1-200
