# A/B timing of one environment switch on one box: bash tools/gpu_ab_env.sh TAG VAR VALUE_A VALUE_B
# [MODE...]: each value runs the C3 line of each mode (train, fwd) twice, in alternating order;
# then tools/bench_summary.py over all logs.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=$1; V=$2; A=$3; B=$4; shift 4
MODES=${*:-train fwd}
for rep in 1 2; do
  for val in $A $B; do
    for m in $MODES; do
      env $V=$val timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 --steps 12 --warmup 3 --mode $m \
        > gpurun_out/${T}_${V}${val}_${m}${rep}.log 2>&1
    done
  done
done
python tools/bench_summary.py gpurun_out/${T}_*.log
