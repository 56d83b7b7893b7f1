set -o pipefail
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
AEROGNN_LIB=aero-gnn_amd/aerognn/libaerognn_prev.so timeout -k 10 300 python -u tools/ab_outputs.py save gpurun_out/ab_prev.pt > gpurun_out/r3m_ab.log 2>&1 && \
timeout -k 10 300 python -u tools/ab_outputs.py save gpurun_out/ab_new.pt >> gpurun_out/r3m_ab.log 2>&1 && \
AEROGNN_LIB=aero-gnn_amd/aerognn/libaerognn_var.so timeout -k 10 300 python -u tools/ab_outputs.py save gpurun_out/ab_var.pt >> gpurun_out/r3m_ab.log 2>&1 && \
python tools/ab_outputs.py cmp gpurun_out/ab_new.pt gpurun_out/ab_prev.pt >> gpurun_out/r3m_ab.log 2>&1 ; \
python tools/ab_outputs.py cmp gpurun_out/ab_var.pt gpurun_out/ab_prev.pt >> gpurun_out/r3m_ab.log 2>&1 ; \
rm -f gpurun_out/ab_*.pt; \
for L in libaerognn libaerognn_var libaerognn_prev; do \
AEROGNN_LIB=aero-gnn_amd/aerognn/$L.so timeout -k 10 300 python -u bench.py --config c5 --mode fwd --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3m_c5_$L.log 2>&1 || exit 1; \
AEROGNN_LIB=aero-gnn_amd/aerognn/$L.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > gpurun_out/r3m_c3_$L.log 2>&1 || exit 1; \
done
