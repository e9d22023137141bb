#!/bin/bash
# Adam histories in the persistent kernel's exit (no k_adam_hist launch)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> gpurun_out/adamtail_steps.txt; return $rc; }
: > gpurun_out/adamtail_steps.txt
run tests timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_status.py tests/test_gpu_restarts.py tests/test_gpu_timeshard.py \
  -k "adam or fit_em or stop or golden or timeout or batched or neuron_sharded or restart" > gpurun_out/adamtail_tests.txt 2>&1 && \
run bench timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/adamtail_bench.json 2> gpurun_out/adamtail_bench.err && \
run prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_adamtail -o run -- python3 bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/adamtail_prof.log 2>&1
