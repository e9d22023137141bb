#!/bin/bash
# C3 bench at several backward chunk lengths (forward chunk 49)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cb in 98 49 66; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --chunk-bwd $cb \
    > gpurun_out/bwd_sweep_$cb.json 2> gpurun_out/bwd_sweep_$cb.err || exit 1
done
