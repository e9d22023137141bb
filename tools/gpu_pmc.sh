# PMC passes for the bench workload (run via gpurun from the repo root).  Each pass is
# its own rocprofv3 run with counters only (no sys/runtime traces).
TAG=${1:-pmc}
CFG=${2:-c3}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "k_ptb3|k_emission_i8|k_emission_yreg|k_emission_pipe|k_adam<|k_forward<|k_backward<|k_verify|k_forward_relax|k_backward_relax" --output-format csv -d $R/gpurun_out/${TAG}_$name -o run \
    -- python3 $R/bench.py --config $CFG --steps 3 --warmup 3 --no-cpu-baseline --no-api-fit > $R/gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; return $rc
}
run fetch FETCH_SIZE && run write WRITE_SIZE && \
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS && \
run sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
