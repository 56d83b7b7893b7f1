# Same-box A/B of library builds on the fused edge backward / edge forward (tools/eb_variants.py):
# bash tools/eb_ab.sh TAG FILTER lib1.so lib2.so ... ("cur" = the in-tree library), three alternations.
set -e
set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
T=$1; F=$2; shift 2
for rep in 1 2 3; do
  for L in "$@" cur; do
    n=$(basename $L .so)
    if [ "$L" = cur ]; then unset AEROGNN_LIB; else export AEROGNN_LIB=$L; fi
    echo "== $n rep $rep"
    timeout -k 10 200 python -u tools/eb_variants.py --reps 20 --only "$F" 2>&1 | grep -v amdgpu.ids | tail -n +2
  done
done
