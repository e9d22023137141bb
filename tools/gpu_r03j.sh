#!/bin/bash
# Round-3 session j: C3 scan warm-up sweep at HEAD (driver window 6-25), default chunks.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for W in 48 40 32 24; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 --warm-steps $W \
    > gpurun_out/r03j_w$W.json 2> gpurun_out/r03j_w$W.err || exit 1
  python3 -c "
import json; b=json.load(open('gpurun_out/r03j_w$W.json'))
k=b['kernels_ms']; r=b['roofline']
print('W=$W', round(b['value'],1), 'it/s frac', round(r['frac'],3), 'fwd', k['forward_filter'], 'frep', k['forward_repair'], 'bwd', k['backward_smoother'], 'brep', k['backward_repair'], 'rep', b['repairs_last'], flush=True)" >> gpurun_out/r03j_sweep.txt
done
