#!/bin/bash
# Round-3 session g: persistent Adam with row blocks (L in (512, 1024]): parity, C3 body time, C4 rehearsal.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_timeshard.py tests/test_gpu_restarts.py -x -v \
  --timeout 200 --timeout-method thread -k "adam or neuron or restart or fit_em" > gpurun_out/r03g_tests.txt 2>&1 &&
timeout -k 10 150 python -u tools/adam_prof.py 512 100000 512 300 > gpurun_out/r03g_adamprof.txt 2>&1 &&
timeout -k 10 150 python -u tools/adam_prof.py 128 20000 1024 300 > gpurun_out/r03g_adamprof_l1024.txt 2>&1 &&
timeout -k 10 400 python -u bench.py --config c4 --shard time --virtual 8 --steps 3 --warmup 1 --no-cpu-baseline \
  --no-api-fit > gpurun_out/r03g_c4_virtual8.json 2> gpurun_out/r03g_c4_virtual8.err
