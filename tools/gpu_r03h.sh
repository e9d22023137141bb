#!/bin/bash
# Round-3 session h: emission kernels (k_emission_pipe, k_emission_yreg): bit-identity vs k_emission_i8, timing, C3 bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "emission" > gpurun_out/r03h_tests.txt 2>&1 &&
timeout -k 10 200 python -u tools/diag_emission.py --out gpurun_out/r03h_emission.json > gpurun_out/r03h_emission.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-api-fit > gpurun_out/r03h_bench.json 2> gpurun_out/r03h_bench.err
PMG_LIB_PATH=exp/emstamp/libpmg_hip.so timeout -k 10 200 python -u tools/diag_emission.py --only yreg --reps 2 \
  > gpurun_out/r03h_yreg_stamps.txt 2>&1
