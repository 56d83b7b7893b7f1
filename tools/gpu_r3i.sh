set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T="python -u -m pytest -v -s --timeout 900 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_bsmsgnn.py > gpurun_out/r3i_bsmsgnn.log 2>&1 ; \
timeout -k 10 900 $T tests/test_gpu_configs.py -k "c5_pooling or c3_full or bf16_vs_fp32" --durations=5 > gpurun_out/r3i_configs.log 2>&1
