set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
R=$PWD
for c in 9352153 7db15f3 314b436 3e6728d; do
  (cd _bisect/$c && timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/r3v_smoke_$c.log 2>&1) ; true
done
