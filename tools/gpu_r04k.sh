#!/bin/bash
# round 4 k: suff-stats with the f64 flush staggered across the two waves of a SIMD
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r04k_steps.txt; return $rc; }
: > gpurun_out/r04k_steps.txt
run tests timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_restarts.py -k "suffstats or fit_em or golden or restart" > gpurun_out/r04k_tests.txt 2>&1 && \
run bench timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04k_bench.json 2> gpurun_out/r04k_bench.err && \
run prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04k -o run -- python3 bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04k_prof.log 2>&1
