# Round-3 final evidence set on the round's last kernels: profile set r3f, then the bench lines
# (the default line reads profiles/r3f_pmc_traffic.json, copied in place first).
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
bash tools/profile_round.sh r3f 3
cp gpurun_out/pmc_traffic_r3f.json profiles/r3f_pmc_traffic.json
timeout -k 10 600 python -u bench.py > gpurun_out/r3f_bench.log 2>&1
AEROGNN_FUSED_EDGE_BWD=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 > gpurun_out/r3f_bench_split.log 2>&1
timeout -k 10 300 python -u bench.py --mode fwd --no-cpu-baseline --no-c4 > gpurun_out/r3f_bench_c3_fwd.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --mode fwd --no-cpu-baseline --no-c4 > gpurun_out/r3f_bench_c5_fwd.log 2>&1
