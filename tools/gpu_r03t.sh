#!/bin/bash
# Round-3 session t: Hilbert metric as log of the ratio -- C5 restarts, C3 bench, GPU suite.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --restarts 8 --no-cpu-baseline --no-api-fit > gpurun_out/r03t_c5.json 2> gpurun_out/r03t_c5.err &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03t_c3.json 2> gpurun_out/r03t_c3.err &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03t_tests.txt 2>&1
