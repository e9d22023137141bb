# quick GPU iteration: parity tests + bench (+ optional Adam phase stamps)
TAG=${1:-q}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_$TAG.log').read().strip().splitlines()[-1])
print('value', round(d['value'],1), 'ms', round(d['ms_per_step'],3), 'fb GB/s', round(d['fwd_bwd_GBps']), 'rep', d['repairs_last'], 'warm', d['scan_warmup_fwd_bwd'])
print(d['kernels_ms'])"
if [ -n "$ADAMPROF" ]; then
  PMG_ADAM_PROF=1 timeout -k 10 200 python bench.py --steps 3 --warmup 3 --no-cpu-baseline > gpurun_out/adamprof_$TAG.log 2>&1; grep "adam prof" gpurun_out/adamprof_$TAG.log | tail -3
fi
