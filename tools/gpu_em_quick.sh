# emission-focused check: emission/EM/decode parity + bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "emission or golden or fit_em or decode or naive" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_emq.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_emq.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_emq.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_emq.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_emq.log').read().strip().splitlines()[-1])
print('value', round(d['value'],1), 'ms', round(d['ms_per_step'],3)); print(d['kernels_ms'])"
