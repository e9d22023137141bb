#!/bin/bash
# round 4 l: decode results through page-locked buffers; buffer cache
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r04l_steps.txt; return $rc; }
: > gpurun_out/r04l_steps.txt
run tests timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_host_buffers.py tests/test_gpu_configs.py tests/test_gpu_shuffle.py tests/test_gpu_dense.py \
  tests/test_gpu_parity.py -k "host or decode or shuffle or dense or c2 or c3 or latentonly or latent_only or api" > gpurun_out/r04l_tests.txt 2>&1 && \
run bench timeout -k 10 400 python -u bench.py --no-cpu-baseline --decode --warmup 5 --steps 20 > gpurun_out/r04l_bench.json 2> gpurun_out/r04l_bench.err
