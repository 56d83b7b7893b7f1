#!/bin/bash
# SQ/TA/TCC counter passes of tools/layer_micro.py (one MGN layer fwd+bwd at C3 fine level).
set -e
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$R"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_VMEM" \
           "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum TD_BUSY_avr"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/ctr_$i -o m -- \
      python tools/layer_micro.py 2 > gpurun_out/ctr_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/ctr_$i.log; }
done
python tools/pmc_summary.py "${KFILTER:-res_kernel|wgrad_kernel|segment_sum}" gpurun_out/ctr_* > gpurun_out/ctr_summary.txt
