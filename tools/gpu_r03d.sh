#!/bin/bash
# Round-3 session d: batched masks (row-walking kernel), emission MT = 1 vs 2 on the C3 bench,
# seeded warm-up study.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model_selection.py tests/test_gpu_shuffle.py -x -v --timeout 200 \
  --timeout-method thread > gpurun_out/r03d_tests.txt 2>&1 &&
for mt in 1 2; do
  PMG_EMISSION_MT=$mt timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-api-fit \
    > gpurun_out/r03d_bench_mt$mt.json 2> gpurun_out/r03d_bench_mt$mt.err || exit 1
done
timeout -k 10 300 python -u tools/bench_extra.py > gpurun_out/r03d_extra.json 2> gpurun_out/r03d_extra.err &&
timeout -k 10 300 python -u tools/diag_seeded_warmup.py 6 > gpurun_out/r03d_seeded.txt 2>&1 &&
timeout -k 10 300 python -u tools/diag_seeded_warmup.py 15 >> gpurun_out/r03d_seeded.txt 2>&1
