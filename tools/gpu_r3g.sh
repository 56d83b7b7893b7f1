set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T="python -u -m pytest -x -v -s --timeout 600 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_fullsize.py -k "c2_layer" > gpurun_out/r3g_c2.log 2>&1
