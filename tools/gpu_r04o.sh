#!/bin/bash
# round 4 o: Adam partial sums by one wave (quad sums in LDS); 8-byte rblk / ll64 stores in the emission
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r04o_steps.txt; return $rc; }
: > gpurun_out/r04o_steps.txt
run tests timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_status.py tests/test_gpu_restarts.py -k "adam or fit_em or stop or golden or timeout or batched or emission" > gpurun_out/r04o_tests.txt 2>&1 && \
run prof timeout -k 10 200 python -u tools/adam_prof.py > gpurun_out/r04o_adamprof.txt 2>&1 && \
run bench timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04o_bench.json 2> gpurun_out/r04o_bench.err && \
run bench2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04o_bench2.json 2> gpurun_out/r04o_bench2.err
