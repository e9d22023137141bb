#!/bin/bash
# Round-3 final (a, after the emission rewrite): full GPU suite, smoke, C3 bench (default window and the driver's window).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r03k_final_tests.txt 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03k_final_smoke.txt 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r03k_final_bench_default.json 2> gpurun_out/r03k_final_bench_default.err &&
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 > gpurun_out/r03k_final_bench_driver.json \
  2> gpurun_out/r03k_final_bench_driver.err
