# Round-4 session s: resident edge forward at 12 / 16 waves per CU (build_ab/libW12.so, libW16.so:
# three / four waves per SIMD, direct e loads, no deferred stores) against the in-tree 8 waves:
# bitwise resident-vs-general tests with each build, then C3 forward and train lines.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=${1:-r4s}
for L in build_ab/libW12.so build_ab/libW16.so; do
  n=$(basename $L .so)
  AEROGNN_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -v -k "resident or fused_edge" \
      --timeout 200 --timeout-method thread > gpurun_out/${T}_${n}_tests.log 2>&1
  tail -1 gpurun_out/${T}_${n}_tests.log
done
for rep in 1 2; do
  for L in cur build_ab/libW12.so build_ab/libW16.so; do
    n=$(basename $L .so)
    if [ "$L" = cur ]; then unset AEROGNN_LIB; else export AEROGNN_LIB=$L; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 --steps 12 --warmup 3 --mode fwd \
        > gpurun_out/${T}_${n}_fwd${rep}.log 2>&1
  done
done
unset AEROGNN_LIB
python tools/bench_summary.py gpurun_out/${T}_*_fwd*.log
