#!/bin/bash
# round 4 final (b): full GPU suite at HEAD, C5 batched restarts, C4 on 8 virtual time shards
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r04jb_steps.txt; return $rc; }
: > gpurun_out/r04jb_steps.txt
run suite timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r04jb_tests.txt 2>&1 && \
run c5 timeout -k 10 300 python -u bench.py --restarts 8 --no-cpu-baseline --no-api-fit --warmup 5 --steps 10 > gpurun_out/r04jb_c5.json 2> gpurun_out/r04jb_c5.err && \
run c4v timeout -k 10 400 python -u bench.py --config c4 --shard time --virtual 8 --no-cpu-baseline --no-api-fit --warmup 2 --steps 3 > gpurun_out/r04jb_c4v8.json 2> gpurun_out/r04jb_c4v8.err
