set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread --durations=10 > gpurun_out/r3t_gpu_tests.log 2>&1 ; \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3t_smoke.log 2>&1
