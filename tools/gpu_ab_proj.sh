# A/B of the projection kernel's single x-tile load (in-tree) against build_ab/libPJ0.so: the
# bitwise projection test first, then the C3 train and forward lines, twice, alternating.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=${1:-r4v}
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -v -k "proj" --timeout 200 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1
tail -1 gpurun_out/${T}_tests.log
bash tools/gpu_ab.sh $T build_ab/libPJ0.so
