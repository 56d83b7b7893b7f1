# Round-4 session m: L2-prefetch variants of the fused edge backward (AGN_EB_PREFETCH 1/2/3) and
# the resident edge forward (AGN_FWD_PREFETCH 1). Bitwise tests on two variants first (a fault
# ends the script), then the A/B timing of all variants against the in-tree build.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=${1:-r4m}
AEROGNN_LIB=build_ab/libE2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -v -k "fused_edge or resident" \
    --timeout 200 --timeout-method thread > gpurun_out/${T}_testE2.log 2>&1
tail -1 gpurun_out/${T}_testE2.log
AEROGNN_LIB=build_ab/libF1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -v -k "fused_edge or resident" \
    --timeout 200 --timeout-method thread > gpurun_out/${T}_testF1.log 2>&1
tail -1 gpurun_out/${T}_testF1.log
bash tools/gpu_ab.sh $T build_ab/libE1.so build_ab/libE2.so build_ab/libE3.so build_ab/libF1.so
