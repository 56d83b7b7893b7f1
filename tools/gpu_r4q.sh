# Round-4 session q: deferred G0 / de stores in the fused edge backward (in-tree, AGN_EB_DEFER=1)
# against build_ab/libB0.so (stores at the tile end): bitwise fused-vs-split and the bf16 oracle
# tests first, then the level-0 launch time and the C3 train line, twice, alternating.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=${1:-r4q}
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_bf16.py -v -rP \
    -k "resident or fused_edge or c2_layer_bf16 or bsms4" --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
grep -E "passed|failed" gpurun_out/${T}_tests.log | tail -1
for rep in 1 2; do
  for L in cur build_ab/libB0.so; do
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
