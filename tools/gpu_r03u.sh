#!/bin/bash
# Round-3 session u (after the Hilbert-metric fix): first-iteration breakdown at three
# warm-ups, smoke, the driver-window C3 bench, and the rocprofv3 kernel stats of the bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/diag_iter1.py --iters 4 --warms 48,128,256 --out gpurun_out/r03u_iter1.jsonl > gpurun_out/r03u_iter1.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03u_smoke.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 > gpurun_out/r03u_bench_driver.json 2> gpurun_out/r03u_bench_driver.err &&
timeout -k 10 200 python -u tools/diag_repairs.py > gpurun_out/r03u_repairs.txt 2>&1 &&
bash tools/gpu_prof.sh r03u c3
