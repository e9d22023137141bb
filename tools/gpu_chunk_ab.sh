#!/bin/bash
# Interleaved bench windows at several scan configurations on one box.
# usage: tools/gpu_chunk_ab.sh OUTDIR "fc,bc[,tw] ..." REPS
#   fc, bc: forward / backward chunk; tw: main-pass chains on two waves (--two-waves)
set -o pipefail
out=$1; cfgs=$2; reps=${3:-2}
mkdir -p "$out"
for r in $(seq 1 "$reps"); do
  for c in $cfgs; do
    IFS=, read -r fc bc tw <<< "$c"
    extra=""; [ "$tw" = "tw" ] && extra="--two-waves"
    tag="c${fc}_${bc}${tw:+_$tw}_r$r"
    timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-api-fit \
      --chunk "$fc" --chunk-bwd "$bc" $extra > "$out/$tag.json" 2> "$out/$tag.err" || exit 1
    python - "$out/$tag.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d['kernels_ms']
print(sys.argv[1], round(d['value'], 1), d['chunk'], d['chunk_bwd'], 'fwd', k['forward_filter'], k['forward_repair'],
      'bwd', k['backward_smoother'], k['backward_repair'], 'rep', d['repairs_last'], 'fresh', round(d['fresh_fit']['em_iters_per_s'], 1),
      'it1', d['fresh_fit']['warmup_iteration_s'][0], 'lml', d['log_marginal_last'], flush=True)
PY
  done
done
