# Round-3 closing check on the final tree (default kernels unchanged since the r3f evidence set):
# the full GPU suite, smoke, and the default bench line.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3s5_gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3s5_smoke.log 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/r3s5_bench.log 2>&1
