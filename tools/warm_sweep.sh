# scan warm-up sweep at C3 (fixed per-pass warm-ups), bench only
for wf in "48,48" "40,40" "32,32" "32,48" "24,32" "40,24" "64,32"; do
  timeout -k 10 200 python bench.py --steps 8 --warmup 3 --no-cpu-baseline --warm-fb $wf > gpurun_out/ws_$wf.log 2>&1 || { echo "fail $wf"; exit 1; }
  tail -1 gpurun_out/ws_$wf.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_ms']; print('$wf', round(d['value'],1), 'fwd', k['forward_filter'], k['forward_repair'], 'bwd', k['backward_smoother'], k['backward_repair'], 'rep', d['repairs_last'])"
done
