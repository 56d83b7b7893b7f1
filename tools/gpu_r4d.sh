set -e
mkdir -p gpurun_out
export AEROGNN_MEMLOG=0
AEROGNN_LIB=build_ab/libA.so timeout -k 10 200 python -u tools/ab_layer.py save gpurun_out/l_A.pt
timeout -k 10 200 python -u tools/ab_layer.py save gpurun_out/l_B.pt
python tools/ab_layer.py cmp gpurun_out/l_A.pt gpurun_out/l_B.pt
rm -f gpurun_out/l_A.pt gpurun_out/l_B.pt
