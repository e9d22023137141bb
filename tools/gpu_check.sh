#!/bin/bash
# focused GPU check of the in-tree library: scan / EM / restart / time-shard tests, then the
# driver-window bench and its rocprof kernel trace (TAG = output prefix)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-chk}
run() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> gpurun_out/${TAG}_steps.txt; return $rc; }
: > gpurun_out/${TAG}_steps.txt
run tests timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_restarts.py tests/test_gpu_timeshard.py tests/test_gpu_configs.py \
  -k "${SEL:-forward or backward or logz or fit_em or restart or golden or c2 or c3 or timeshard or masked}" > gpurun_out/${TAG}_tests.txt 2>&1 && \
run bench timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && \
run prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/${TAG}_prof.log 2>&1
