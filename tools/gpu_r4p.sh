# Round-4 session p: deferred e' stores in the resident edge forward (in-tree, AGN_FWD_DEFER=1)
# against build_ab/libD0.so (stores at the tile end) and libNS.so (stores suppressed: diagnostic):
# bitwise tests first, then C3 forward lines, twice, alternating.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=${1:-r4p}
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -v -k "resident or fused_edge" --timeout 200 \
    --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
tail -1 gpurun_out/${T}_tests.log
for rep in 1 2; do
  for L in cur build_ab/libD0.so build_ab/libNS.so; do
    n=$(basename $L .so)
    if [ "$L" = cur ]; then unset AEROGNN_LIB; else export AEROGNN_LIB=$L; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 --steps 12 --warmup 3 --mode fwd \
        > gpurun_out/${T}_${n}_fwd${rep}.log 2>&1
  done
done
unset AEROGNN_LIB
python tools/bench_summary.py gpurun_out/${T}_*_fwd*.log
