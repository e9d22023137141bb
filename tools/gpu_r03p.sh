#!/bin/bash
# Round-3 session p: softplus tuning with 8 rows per thread: bit-identity vs the row-wise kernel, EM parity, A/B bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread \
  -k "softplus or em_ or golden or c3 or c5 or adam" > gpurun_out/r03p_tests.txt 2>&1 &&
PMG_SOFTPLUS_ROWWISE=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r03p_bench_rowwise.json 2> gpurun_out/r03p_bench_rowwise.err &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r03p_bench_rows8.json 2> gpurun_out/r03p_bench_rows8.err
