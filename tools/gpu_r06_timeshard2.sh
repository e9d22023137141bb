#!/bin/bash
# round 6: time-shard benches with the uninstrumented timed window (C4 8 virtual shards,
# C3 over RCCL at world 1 next to the default engine) and the time-shard GPU tests
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --config c4 --shard time --virtual 8 --no-cpu-baseline --warmup 2 --steps 5 > $O/c4v8.json 2> $O/c4v8.err && \
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 bench.py --shard time --no-cpu-baseline --warmup 5 --steps 20 > $O/c3_time_w1.json 2> $O/c3_time_w1.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > $O/c3_default.json 2> $O/c3_default.err && \
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29562 bench.py --shard time --no-cpu-baseline --warmup 5 --steps 20 > $O/c3_time_w1_b.json 2> $O/c3_time_w1_b.err && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_timeshard.py tests/test_gpu_nccl.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
