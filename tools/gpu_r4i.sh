set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=${1:-r4i}
timeout -k 10 200 python -u tools/wgrad_we_micro.py > gpurun_out/${T}_wgrad_we.txt 2>&1 || true
cat gpurun_out/${T}_wgrad_we.txt | grep -v amdgpu
timeout -k 10 200 python -u tools/edge_bwd_stamps.py > gpurun_out/${T}_ebtime.txt 2>&1 || true
head -2 gpurun_out/${T}_ebtime.txt | grep -v amdgpu
bash tools/gpu_r4g.sh $T
