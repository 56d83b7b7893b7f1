set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
for rep in 1 2; do for L in libaerognn libaerognn_v1; do \
AEROGNN_LIB=aero-gnn_amd/aerognn/$L.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > gpurun_out/r3aa_${L}_$rep.log 2>&1 || exit 1; \
done; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "res or proj or fwd or forward" > gpurun_out/r3aa_tests.log 2>&1
