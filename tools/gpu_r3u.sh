set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3u_smoke.log 2>&1 ; \
AEROGNN_LIB=aero-gnn_amd/aerognn/libaerognn_prev.so timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3u_smoke_prev.log 2>&1 ; \
true
