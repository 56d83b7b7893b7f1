# The GPU suite, the smoke check and the default bench line on this tree.
# pytest exit 1 (test failures) continues to the smoke and the bench; any other non-zero status
# (a crash, an abort, a time limit) ends the script.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=${1:-r4a}
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_gpu_tests.log 2>&1 || rc=$?
tail -3 gpurun_out/${T}_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests ended with status $rc"; exit $rc; fi
grep -q "Memory access fault\|Fatal Python error\|core dumped" gpurun_out/${T}_gpu_tests.log && exit 3
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
tail -2 gpurun_out/${T}_smoke.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.log 2>&1
tail -1 gpurun_out/${T}_bench.log | cut -c1-400
