#!/bin/bash
# Round-3 session b: batched masks / shuffles parity, their timing, Adam body vs neurons per workgroup.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_model_selection.py tests/test_gpu_shuffle.py tests/test_gpu_parity.py \
  -x -v --timeout 200 --timeout-method thread > gpurun_out/r03b_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/bench_extra.py > gpurun_out/r03b_extra.json 2> gpurun_out/r03b_extra.err &&
for n in 256 1024; do
  timeout -k 10 150 python -u tools/adam_prof.py $n 100000 512 300 > gpurun_out/r03b_adamprof_n$n.txt 2>&1 || exit 1
done
# cooperative vs plain launches of the persistent kernels (driver window)
for mode in coop plain; do
  if [ $mode = plain ]; then export PMG_NO_COOP=1; else unset PMG_NO_COOP; fi
  timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-api-fit \
    > gpurun_out/r03b_bench_$mode.json 2> gpurun_out/r03b_bench_$mode.err || exit 1
done
