#!/bin/bash
# C3 bench at several scan warm-ups (the relaxation repairs whatever a short warm-up misses)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for W in 48 32 24 16; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warm-steps $W > gpurun_out/warm_$W.json 2> gpurun_out/warm_$W.err || exit 1
  python3 -c "
import json; b=json.load(open('gpurun_out/warm_$W.json'))
k=b['kernels_ms']; print('W=$W', round(b['value'],1), 'it/s', 'fwd', k['forward_filter'], 'frep', k['forward_repair'], 'bwd', k['backward_smoother'], 'brep', k['backward_repair'], 'fresh_fit_s', round(b['fresh_fit']['device_s'],4), 'repairs_last', b['repairs_last'])"
done
