# Round-3 closing check after the two-rows-in-flight node walk (AGN_WALK2):
# the full GPU suite, smoke, and the default bench line.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3s7_gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3s7_smoke.log 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/r3s7_bench.log 2>&1
