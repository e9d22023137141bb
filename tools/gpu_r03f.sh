#!/bin/bash
# Round-3 session f: Adam without in-loop spills (LDS constants, uniform bias index): body time, parity, bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 python -u tools/adam_prof.py 512 100000 512 300 > gpurun_out/r03f_adamprof.txt 2>&1 &&
timeout -k 10 150 python -u tools/adam_prof.py 1024 100000 512 300 > gpurun_out/r03f_adamprof_n1024.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_restarts.py tests/test_gpu_timeshard.py -x -v \
  --timeout 200 --timeout-method thread -k "adam or fit_em or restart or neuron or emission" > gpurun_out/r03f_tests.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-api-fit \
  > gpurun_out/r03f_bench.json 2> gpurun_out/r03f_bench.err
