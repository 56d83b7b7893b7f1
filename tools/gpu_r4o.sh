# Round-4 session o: diagnostic timing with the edge kernels' output stores suppressed
# (build_ab/libNS.so, -DAGN_EB_NOSTORE -DAGN_FWD_NOSTORE): how much of a tile waits on stores.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=${1:-r4o}
for rep in 1 2; do
  for L in cur build_ab/libNS.so; do
    n=$(basename $L .so)
    if [ "$L" = cur ]; then unset AEROGNN_LIB; else export AEROGNN_LIB=$L; fi
    rc=0
    timeout -k 10 200 python -u tools/edge_bwd_stamps.py > gpurun_out/${T}_${n}_eb${rep}.txt 2>&1 || rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "timing ended with status $rc"; exit $rc; fi
    grep "per launch" gpurun_out/${T}_${n}_eb${rep}.txt | sed "s/^/$n: /"
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 --steps 12 --warmup 3 --mode fwd \
        > gpurun_out/${T}_${n}_fwd${rep}.log 2>&1
  done
done
unset AEROGNN_LIB
python tools/bench_summary.py gpurun_out/${T}_*_fwd*.log
