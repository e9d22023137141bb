#!/bin/bash
# Round-3 session v: C4 8-virtual-shard rehearsal on one GPU after the Hilbert-metric fix.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --config c4 --shard time --virtual 8 --steps 3 --warmup 1 --no-cpu-baseline \
  --no-api-fit > gpurun_out/r03v_c4_virtual8.json 2> gpurun_out/r03v_c4_virtual8.err
