# A/B timing of library builds on one box: bash tools/gpu_ab.sh TAG lib1.so lib2.so ... (the in-tree
# libaerognn.so is "cur"); each build runs the C3 train line and the C3 forward-only line, twice,
# in alternating order; then tools/bench_summary.py over all logs.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=$1; shift
B="bench.py --no-cpu-baseline --no-c4 --steps 12 --warmup 3"
for rep in 1 2; do
  for L in "$@" cur; do
    n=$(basename $L .so)
    if [ "$L" = cur ]; then unset AEROGNN_LIB; else export AEROGNN_LIB=$L; fi
    timeout -k 10 300 python -u $B > gpurun_out/${T}_${n}_train${rep}.log 2>&1
    timeout -k 10 300 python -u $B --mode fwd > gpurun_out/${T}_${n}_fwd${rep}.log 2>&1
  done
done
unset AEROGNN_LIB
python tools/bench_summary.py gpurun_out/${T}_*_train*.log gpurun_out/${T}_*_fwd*.log
