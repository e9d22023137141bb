# time-shard GPU check: parity tests + C4 bench (1 shard and 8 virtual shards on one GPU)
TAG=${1:-ts}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_timeshard.py tests/test_gpu_parity.py -k "timeshard or adam" -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_ts_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_ts_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --shard time --config c4 --steps 5 --warmup 2 > gpurun_out/bench_c4_1_$TAG.log 2>&1 || { echo "c4 bench failed"; tail -20 gpurun_out/bench_c4_1_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_c4_1_$TAG.log | cut -c1-700
timeout -k 10 400 python -u bench.py --shard time --config c4 --virtual 8 --steps 5 --warmup 2 > gpurun_out/bench_c4_v8_$TAG.log 2>&1 || { echo "c4 v8 bench failed"; tail -20 gpurun_out/bench_c4_v8_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_c4_v8_$TAG.log | cut -c1-700
