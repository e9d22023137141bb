#!/bin/bash
# C3 bench over (scan warm-up W, forward chunk C, backward chunk Cb): in steady state the
# sharp emission makes chains forget within a few steps, so short warm-ups + more, shorter
# chunks trade main-pass work against rare relaxation repairs.  Driver window (5 + 20).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-r03}
for W in ${WS:-48 16 8 4}; do
 for cfg in ${CFGS:-49:98 32:64 25:50 25:100}; do
  C=${cfg%:*}; CB=${cfg#*:}
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 --warm-steps $W \
    --chunk $C --chunk-bwd $CB > gpurun_out/sw_${TAG}_${W}_${C}_${CB}.json 2> gpurun_out/sw_${TAG}_${W}_${C}_${CB}.err || exit 1
  python3 -c "
import json; b=json.load(open('gpurun_out/sw_${TAG}_${W}_${C}_${CB}.json'))
k=b['kernels_ms']; r=b['roofline']
print('W=$W C=$C Cb=$CB', round(b['value'],1), 'it/s frac', round(r['frac'],3), 'fwd', k['forward_filter'], 'frep', k['forward_repair'], 'bwd', k['backward_smoother'], 'brep', k['backward_repair'], 'fresh', round(b['fresh_fit']['device_s'],4), 'rep', b['repairs_last'], flush=True)"
 done
done
