# Round-4 session u: the fused backward waits for its re-read g / dAgg rows before the G0 stores
# issue (in-tree) against build_ab/libP0.so (without): bitwise tests, then the level-0 launch and
# the C3 train line, twice, alternating.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=${1:-r4u}
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_bf16.py -v -rP \
    -k "fused_edge or c2_layer_bf16" --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
grep -E "passed|failed" gpurun_out/${T}_tests.log | tail -1
for rep in 1 2; do
  for L in cur build_ab/libP0.so; do
    n=$(basename $L .so)
    if [ "$L" = cur ]; then unset AEROGNN_LIB; else export AEROGNN_LIB=$L; fi
    rc=0
    timeout -k 10 200 python -u tools/edge_bwd_stamps.py > gpurun_out/${T}_${n}_eb${rep}.txt 2>&1 || rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "timing ended with status $rc"; exit $rc; fi
    grep "per launch" gpurun_out/${T}_${n}_eb${rep}.txt | sed "s/^/$n: /"
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 --steps 12 --warmup 3 > gpurun_out/${T}_${n}_train${rep}.log 2>&1
  done
done
unset AEROGNN_LIB
python tools/bench_summary.py gpurun_out/${T}_*_train*.log
