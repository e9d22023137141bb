#!/bin/bash
# Round-3 session l: k_ptb3 with 64 x 256 tiles (default) vs 128 x 128 (PMG_SS_TM=128): parity tests, A/B bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread \
  -k "suffstats or em_ or golden or c5 or restart or adam" > gpurun_out/r03l_tests.txt 2>&1 &&
PMG_SS_TM=128 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r03l_bench_tm128.json 2> gpurun_out/r03l_bench_tm128.err &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r03l_bench_tm64.json 2> gpurun_out/r03l_bench_tm64.err &&
PMG_SS_TM=128 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r03l_bench_tm128b.json 2> gpurun_out/r03l_bench_tm128b.err &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r03l_bench_tm64b.json 2> gpurun_out/r03l_bench_tm64b.err
