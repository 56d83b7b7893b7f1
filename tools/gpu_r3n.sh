set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread --durations=15 > gpurun_out/r3n_gpu_tests.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_concat_r3n -o concat -- \
    python tools/concat_trace.py > gpurun_out/prof_concat_r3n.log 2>&1
