#!/bin/bash
# Round-3 session q: wave-specialised suff-stats (k_ptb3s) vs k_ptb3 (PMG_SS_LEGACY=1): parity + A/B bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread \
  -k "suffstats or em_ or golden or c3 or c5 or c2 or adam" > gpurun_out/r03q_tests.txt 2>&1
echo "tests rc=$?" >> gpurun_out/r03q_tests.txt
PMG_SS_LEGACY=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r03q_bench_legacy.json 2> gpurun_out/r03q_bench_legacy.err &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r03q_bench_spec.json 2> gpurun_out/r03q_bench_spec.err
