#!/bin/bash
# PMC passes (SQ counters only) for the emission and suff-stats kernels of the C3 bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmcem}
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "k_emission_yreg|k_ptb3" --output-format csv -d gpurun_out/${TAG}_$name -o run \
    -- python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --no-api-fit > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc" >> gpurun_out/${TAG}_steps.txt; return $rc
}
: > gpurun_out/${TAG}_steps.txt
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS && \
run sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS && \
run sq3 SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT && \
run wr WRITE_SIZE
