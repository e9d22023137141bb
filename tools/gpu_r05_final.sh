#!/bin/bash
# round-5 closing evidence: smoke, default and driver-window bench lines (with decode), the
# rocprofv3 kernel trace of the driver window, C5 restarts and C4 virtual time shards
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05f_smoke.txt 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r05f_default.json 2> gpurun_out/r05f_default.err && \
timeout -k 10 600 python -u bench.py --warmup 5 --steps 20 --decode > gpurun_out/r05f_window.json 2> gpurun_out/r05f_window.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r05f -o run -- python3 bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r05f_prof.log 2>&1 && \
timeout -k 10 300 python -u bench.py --restarts 8 --no-cpu-baseline > gpurun_out/r05f_c5.json 2> gpurun_out/r05f_c5.err && \
timeout -k 10 500 python -u bench.py --config c4 --shard time --virtual 8 --no-cpu-baseline --warmup 2 --steps 5 > gpurun_out/r05f_c4v8.json 2> gpurun_out/r05f_c4v8.err
