#!/bin/bash
# round 4 f: fit_em returns through pmg_host_alloc buffers reserved up front
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r04f_steps.txt; return $rc; }
: > gpurun_out/r04f_steps.txt
run api timeout -k 10 300 python -u tools/api_fit_profile.py > gpurun_out/r04f_api_profile.json 2> gpurun_out/r04f_api_profile.err && \
run tests timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_configs.py -k "fit_em or golden or api or c1 or c2 or save" > gpurun_out/r04f_tests.txt 2>&1
