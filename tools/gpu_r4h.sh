set -e
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
timeout -k 10 200 python -u tools/edge_bwd_stamps.py > gpurun_out/r4h_cur.txt 2>&1 || true
head -1 gpurun_out/r4h_cur.txt
AEROGNN_LIB=build_ab/libNR.so timeout -k 10 200 python -u tools/edge_bwd_stamps.py > gpurun_out/r4h_noring.txt 2>&1 || true
head -1 gpurun_out/r4h_noring.txt
AEROGNN_LIB=aero-gnn_amd/aerognn/libaerognn_stamps.so timeout -k 10 200 python -u tools/edge_bwd_stamps.py > gpurun_out/r4h_stamps.txt 2>&1
tail -24 gpurun_out/r4h_stamps.txt
