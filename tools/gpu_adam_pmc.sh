#!/bin/bash
# k_adam instruction mix (PMC, three counter passes) over controlled 300-body M-steps at C3 (tools/adam_prof.py); summary: profiles/<round>_adam_pmc_c3.json
# usage: OUT=r05i bash tools/gpu_adam_pmc.sh  (outputs under gpurun_out/$OUT)
set -o pipefail
OUT=${OUT:-r04i}
mkdir -p gpurun_out/$OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU \
  --output-format csv -d gpurun_out/$OUT/p1 -o run -- python3 tools/adam_prof.py > gpurun_out/$OUT/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32 \
  --output-format csv -d gpurun_out/$OUT/p2 -o run -- python3 tools/adam_prof.py > gpurun_out/$OUT/p2.log 2>&1
echo "rc=$?" >> gpurun_out/$OUT/p2.log
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_SMEM \
  --output-format csv -d gpurun_out/$OUT/p3 -o run -- python3 tools/adam_prof.py > gpurun_out/$OUT/p3.log 2>&1
echo "rc=$?" >> gpurun_out/$OUT/p3.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
  --output-format csv -d gpurun_out/$OUT/p4 -o run -- python3 tools/adam_prof.py > gpurun_out/$OUT/p4.log 2>&1
echo "rc=$?" >> gpurun_out/$OUT/p4.log
