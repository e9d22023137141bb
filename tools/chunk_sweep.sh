# scan chunk-length sweep at C3 (adaptive warm-up), bench only
for ch in 49 64 80 98 128; do
  timeout -k 10 200 python bench.py --steps 8 --warmup 4 --no-cpu-baseline --chunk $ch > gpurun_out/cs_$ch.log 2>&1 || { echo "fail $ch"; exit 1; }
  tail -1 gpurun_out/cs_$ch.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_ms']; print('$ch', round(d['value'],1), 'fwd', k['forward_filter'], k['forward_repair'], 'bwd', k['backward_smoother'], k['backward_repair'], 'rep', d['repairs_last'], 'warm', d['scan_warmup_fwd_bwd'])"
done
