#!/bin/bash
# small-kernel consolidation: tuning (8 rows per thread) and one y_w / t_w reduction launch
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> gpurun_out/smallk_steps.txt; return $rc; }
: > gpurun_out/smallk_steps.txt
run tests timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_restarts.py tests/test_gpu_configs.py -k "suffstats or fit_em or restart or tuning or c2 or golden" > gpurun_out/smallk_tests.txt 2>&1 && \
run bench timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/smallk_bench.json 2> gpurun_out/smallk_bench.err && \
run prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_smallk -o run -- python3 bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/smallk_prof.log 2>&1
