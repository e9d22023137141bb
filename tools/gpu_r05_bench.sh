#!/bin/bash
# round-5 evidence, part 2: default and driver-window bench lines, rocprof kernel stats of the
# driver window, C5 restarts and C4 virtual time shards
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/r05_c3_bench_default.json 2> gpurun_out/r05_c3_bench_default.err && \
timeout -k 10 600 python -u bench.py --warmup 5 --steps 20 --decode > gpurun_out/r05_c3_bench_driver_window.json 2> gpurun_out/r05_c3_bench_driver_window.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r05 -o run -- python3 bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r05_prof.log 2>&1 && \
timeout -k 10 300 python -u bench.py --restarts 8 --no-cpu-baseline > gpurun_out/r05_c5_restarts_bench.json 2> gpurun_out/r05_c5.err && \
timeout -k 10 500 python -u bench.py --config c4 --shard time --virtual 8 --no-cpu-baseline --warmup 2 --steps 5 > gpurun_out/r05_c4_virtual8_1gpu.json 2> gpurun_out/r05_c4.err
