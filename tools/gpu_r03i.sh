#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PMG_LIB_PATH=exp/emstamp/libpmg_hip.so timeout -k 10 200 python -u tools/diag_emission.py --only yreg --reps 2 \
  > gpurun_out/r03i_yreg.txt 2>&1
