#!/bin/bash
# Round-3 session m: bench with the measured fit uninstrumented (events in a second fit): both windows.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-api-fit > gpurun_out/r03m_bench_driver.json 2> gpurun_out/r03m_bench_driver.err &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit > gpurun_out/r03m_bench_default.json 2> gpurun_out/r03m_bench_default.err
