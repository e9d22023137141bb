#!/bin/bash
# Round-3 session c: full GPU suite at the working tree, Adam body (LDS ring / LDS bias table vs
# the r03 HEAD kernel), emission MT = 1 vs 2 on the C3 bench, batched-mask timing.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r03c_tests.txt 2>&1 &&
timeout -k 10 150 python -u tools/adam_prof.py 512 100000 512 300 > gpurun_out/r03c_adamprof_new.txt 2>&1 &&
PMG_LIB_PATH=exp/adam_v0/libpmg_hip.so timeout -k 10 150 python -u tools/adam_prof.py 512 100000 512 300 \
  > gpurun_out/r03c_adamprof_v0.txt 2>&1 &&
for mt in 1 2; do
  PMG_EMISSION_MT=$mt timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-api-fit \
    > gpurun_out/r03c_bench_mt$mt.json 2> gpurun_out/r03c_bench_mt$mt.err || exit 1
done
timeout -k 10 300 python -u tools/bench_extra.py > gpurun_out/r03c_extra.json 2> gpurun_out/r03c_extra.err
