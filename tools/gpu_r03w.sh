#!/bin/bash
# Round-3 session w: C4 on one GPU (one time shard, T = 1e6) after the Hilbert-metric fix.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --config c4 --shard time --steps 5 --warmup 1 --no-cpu-baseline \
  --no-api-fit > gpurun_out/r03w_c4_1gpu.json 2> gpurun_out/r03w_c4_1gpu.err
