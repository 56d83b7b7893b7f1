#!/bin/bash
# Collect the round's evidence on the GPU box (run via gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats of bench.py (C3)         -> gpurun_out/prof_$TAG
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE), kernel trace only -> gpurun_out/pmc_{fetch,write}_$TAG
#   3. tools/pmc_traffic.py -> gpurun_out/pmc_traffic_$TAG.json (per launch and per step)
#   4. the same two PMC passes on the split edge backward (AEROGNN_FUSED_EDGE_BWD=0)
#   5. one MFMA-busy pass (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE) -> mfma_$TAG.json
#   6. one stall pass (wave cycles split into waiting / issue-blocked / issuing) -> sq_$TAG.json
#   7. the concat edge-MLP layer's kernel trace (no torch kernels) -> prof_concat_$TAG
# Every GPU step has its own time limit; the script stops at the first failure.
set -e
TAG=${1:-r3e}
STEPS=${2:-3}
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$R"
B="bench.py --no-cpu-baseline --no-c4"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o c3 -- \
    python $B --steps $STEPS --warmup 1 > gpurun_out/prof_$TAG.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$TAG -o c3 -- \
    python $B --steps 1 --warmup 1 > gpurun_out/pmc_fetch_$TAG.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$TAG -o c3 -- \
    python $B --steps 1 --warmup 1 > gpurun_out/pmc_write_$TAG.log 2>&1
# 3 steps per PMC run: 1 warm-up, 1 timed, 1 instrumented (bench.py --profile-steps 1)
python tools/pmc_traffic.py gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG gpurun_out/pmc_traffic_$TAG.json 3
AEROGNN_FUSED_EDGE_BWD=0 timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv \
    -d gpurun_out/pmc_fetch_split_$TAG -o c3 -- python $B --steps 1 --warmup 1 > gpurun_out/pmc_fetch_split_$TAG.log 2>&1
AEROGNN_FUSED_EDGE_BWD=0 timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv \
    -d gpurun_out/pmc_write_split_$TAG -o c3 -- python $B --steps 1 --warmup 1 > gpurun_out/pmc_write_split_$TAG.log 2>&1
python tools/pmc_traffic.py gpurun_out/pmc_fetch_split_$TAG gpurun_out/pmc_write_split_$TAG \
    gpurun_out/pmc_traffic_split_$TAG.json 3
timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
    -d gpurun_out/pmc_mfma_$TAG -o c3 -- python $B --steps 1 --warmup 1 > gpurun_out/pmc_mfma_$TAG.log 2>&1
python tools/mfma_busy.py gpurun_out/pmc_mfma_$TAG gpurun_out/mfma_$TAG.json
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc_sq_$TAG -o c3 -- python $B --steps 1 --warmup 1 \
    > gpurun_out/pmc_sq_$TAG.log 2>&1
python tools/sq_stall.py gpurun_out/pmc_sq_$TAG gpurun_out/sq_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_concat_$TAG -o concat -- \
    python tools/concat_trace.py > gpurun_out/prof_concat_$TAG.log 2>&1
