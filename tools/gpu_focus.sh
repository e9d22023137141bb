#!/bin/bash
# focused GPU check: selected test files (FILES, -k SEL), then the full bench line (api fit
# included) and a rocprof kernel trace of the driver-window bench.  TAG = output prefix.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-focus}
: > gpurun_out/${TAG}_steps.txt
run() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> gpurun_out/${TAG}_steps.txt; return $rc; }
run tests timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  ${FILES:-tests/test_gpu_parity.py} ${SEL:+-k "$SEL"} > gpurun_out/${TAG}_tests.txt 2>&1 && \
run bench timeout -k 10 300 python -u bench.py --no-cpu-baseline --warmup 5 --steps 20 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && \
run prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/${TAG}_prof.log 2>&1
