#!/bin/bash
# round 4 d: f64 softplus/log in the Adam loss, planes off by default, C4 at 150 bodies
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r04d_steps.txt; return $rc; }
: > gpurun_out/r04d_steps.txt
run parity timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "adam or fit_em or golden or planes or suffstats or stop" > gpurun_out/r04d_tests.txt 2>&1 && \
run c4 timeout -k 10 700 python -u -m pytest -x -v -s --timeout 650 --timeout-method thread \
  tests/test_gpu_configs.py::test_c4_time_sharded_vs_single tests/test_gpu_configs.py::test_c5_restarts \
  tests/test_gpu_timeshard.py > gpurun_out/r04d_c4.txt 2>&1 && \
run bench timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04d_bench.json 2> gpurun_out/r04d_bench.err && \
run prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04d -o run -- python3 bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04d_prof.log 2>&1
