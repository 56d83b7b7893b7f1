set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
for L in libaerognn_v2 libaerognn; do \
AEROGNN_LIB=aero-gnn_amd/aerognn/$L.so timeout -k 10 300 python -u tools/ab_outputs.py save gpurun_out/ab_$L.pt > gpurun_out/r3ae_ab_$L.log 2>&1 || exit 1; done
python tools/ab_outputs.py cmp gpurun_out/ab_libaerognn_v2.pt gpurun_out/ab_libaerognn.pt > gpurun_out/r3ae_cmp.log 2>&1
rm -f gpurun_out/ab_*.pt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "node or mean or layer or mgn or bsms or parity" > gpurun_out/r3ae_tests.log 2>&1 || exit 1
for rep in 1 2; do for L in libaerognn_v2 libaerognn; do \
AEROGNN_LIB=aero-gnn_amd/aerognn/$L.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > gpurun_out/r3ae_${L}_$rep.log 2>&1 || exit 1; \
done; done
for L in libaerognn_v2 libaerognn; do \
AEROGNN_LIB=aero-gnn_amd/aerognn/$L.so timeout -k 10 300 python -u bench.py --config c5 --mode fwd --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > gpurun_out/r3ae_c5_${L}.log 2>&1 || exit 1; \
done
