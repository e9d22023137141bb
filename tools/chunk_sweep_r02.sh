#!/bin/bash
# C3 bench at several chunk lengths (forward chunk / backward chunk)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in "49 98" "49 128" "49 196" "64 128" "40 98"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --chunk $1 --chunk-bwd $2 \
    > gpurun_out/chunk_r02_$1_$2.json 2> gpurun_out/chunk_r02_$1_$2.err || exit 1
done
