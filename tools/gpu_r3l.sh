set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
AEROGNN_LIB=aero-gnn_amd/aerognn/libaerognn_stamps.so timeout -k 10 300 python -u tools/fwd_stamps.py > gpurun_out/r3l_fwd_stamps.log 2>&1
