#!/bin/bash
# round 4 n: k_ptb3 with register double-buffered MFMA operands
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r04n_steps.txt; return $rc; }
: > gpurun_out/r04n_steps.txt
run tests timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_restarts.py -k "suffstats or fit_em_one or restart" > gpurun_out/r04n_tests.txt 2>&1 && \
run bench timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04n_bench.json 2> gpurun_out/r04n_bench.err && \
run bench2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04n_bench2.json 2> gpurun_out/r04n_bench2.err
