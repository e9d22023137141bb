#!/bin/bash
# round 4 j: table log softplus in k_adam
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r04j_steps.txt; return $rc; }
: > gpurun_out/r04j_steps.txt
run adam timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_status.py tests/test_gpu_restarts.py -k "adam or fit_em or stop or golden or timeout or batched" > gpurun_out/r04j_tests.txt 2>&1 && \
run ts timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread \
  tests/test_gpu_timeshard.py -k "neuron_sharded" > gpurun_out/r04j_ts.txt 2>&1 && \
run prof timeout -k 10 200 python -u tools/adam_prof.py > gpurun_out/r04j_adamprof.txt 2>&1 && \
run bench timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04j_bench.json 2> gpurun_out/r04j_bench.err
