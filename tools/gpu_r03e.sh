#!/bin/bash
# Round-3 session e: batched-mask kernel v3 + emission tile invariance tests; suff-stats early-load A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model_selection.py tests/test_gpu_parity.py -x -v --timeout 200 \
  --timeout-method thread -k "mask or emission" > gpurun_out/r03e_tests.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-api-fit \
  > gpurun_out/r03e_bench_base.json 2> gpurun_out/r03e_bench_base.err &&
PMG_LIB_PATH=exp/ss_early/libpmg_hip.so timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --no-cpu-baseline \
  --no-api-fit > gpurun_out/r03e_bench_ssearly.json 2> gpurun_out/r03e_bench_ssearly.err &&
timeout -k 10 300 python -u tools/bench_extra.py > gpurun_out/r03e_extra.json 2> gpurun_out/r03e_extra.err
