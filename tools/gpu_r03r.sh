#!/bin/bash
# Round-3 session r: C5 batched restarts and the C4 8-shard single-GPU rehearsal at HEAD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --restarts 8 --no-cpu-baseline --no-api-fit > gpurun_out/r03r_c5_restarts.json 2> gpurun_out/r03r_c5_restarts.err &&
timeout -k 10 500 python -u bench.py --config c4 --shard time --virtual 8 --steps 3 --warmup 1 --no-cpu-baseline \
  --no-api-fit > gpurun_out/r03r_c4_virtual8.json 2> gpurun_out/r03r_c4_virtual8.err
