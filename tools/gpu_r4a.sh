# Round-4 session a: the GPU suite, the smoke check and the default bench line on this tree.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=${1:-r4a}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_gpu_tests.log 2>&1 || echo "gpu tests failed: see gpurun_out/${T}_gpu_tests.log"
grep -q "Fatal Python error\|core dumped\|Segmentation" gpurun_out/${T}_gpu_tests.log && exit 3
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.log 2>&1
tail -1 gpurun_out/${T}_bench.log | cut -c1-300
