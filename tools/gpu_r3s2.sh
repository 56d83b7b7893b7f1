# Session r3s2: node aggregation as a separate segment-sum launch (AEROGNN_NODE_PRESUM) vs the
# node kernel's in-kernel walk: C3 train and C5 forward A/B, plus a bitwise check of a C3 step.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 > gpurun_out/r3s2_bench_base.log 2>&1
AEROGNN_NODE_PRESUM=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 > gpurun_out/r3s2_bench_presum.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --mode fwd --no-cpu-baseline --no-c4 > gpurun_out/r3s2_c5_base.log 2>&1
AEROGNN_NODE_PRESUM=1 timeout -k 10 300 python -u bench.py --config c5 --mode fwd --no-cpu-baseline --no-c4 > gpurun_out/r3s2_c5_presum.log 2>&1
timeout -k 10 200 python -u tools/ab_outputs.py save gpurun_out/r3s2_a.pt > gpurun_out/r3s2_ab.log 2>&1
AEROGNN_NODE_PRESUM=1 timeout -k 10 200 python -u tools/ab_outputs.py save gpurun_out/r3s2_b.pt >> gpurun_out/r3s2_ab.log 2>&1
timeout -k 10 200 python -u tools/ab_outputs.py cmp gpurun_out/r3s2_a.pt gpurun_out/r3s2_b.pt >> gpurun_out/r3s2_ab.log 2>&1
rm -f gpurun_out/r3s2_a.pt gpurun_out/r3s2_b.pt
