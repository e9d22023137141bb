#!/bin/bash
# Round-3 session n: full GPU suite + smoke at HEAD (bench: uninstrumented measured fit).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r03n_tests.txt 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03n_smoke.txt 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r03n_bench_default.json 2> gpurun_out/r03n_bench_default.err &&
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 > gpurun_out/r03n_bench_driver.json 2> gpurun_out/r03n_bench_driver.err
