set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -k "poolmgn or segment_sum" -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/r3o_tests.log 2>&1 ; \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_concat_r3o -o concat -- \
    python tools/concat_trace.py > gpurun_out/prof_concat_r3o.log 2>&1
