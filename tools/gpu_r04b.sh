#!/bin/bash
# round 4 b: full GPU suite (planes between backward and statistics, Adam softplus, new
# parity tests), then the C3 bench (driver window) and a kernel-trace profile of it
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > gpurun_out/r04b_tests.txt 2>&1
echo "tests rc=$?" >> gpurun_out/r04b_tests.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04b -o run -- python3 bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04b_prof.log 2>&1
timeout -k 10 300 python -u tools/api_fit_profile.py > gpurun_out/r04b_api_profile.json 2> gpurun_out/r04b_api_profile.err
