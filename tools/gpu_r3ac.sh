set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
for rep in 1 2; do for L in libaerognn libaerognn_v1; do \
AEROGNN_LIB=aero-gnn_amd/aerognn/$L.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > gpurun_out/r3ac_${L}_$rep.log 2>&1 || exit 1; \
AEROGNN_LIB=aero-gnn_amd/aerognn/$L.so timeout -k 10 300 python -u bench.py --config c5 --mode fwd --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > gpurun_out/r3ac_c5_${L}_$rep.log 2>&1 || exit 1; \
done; done
