#!/bin/bash
# library A/B (V = variant .so, TAG = output prefix): variant tests, then rocprof of the driver-window bench, base vs variant
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> gpurun_out/${TAG:-embpf}_steps.txt; return $rc; }
: > gpurun_out/${TAG:-embpf}_steps.txt
V=${V:-exp/bpf/libpmg_hip.so}
run tests env PMG_LIB_PATH=$V timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_restarts.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py -k "${SEL:-suffstats or planes or fit_em or restart or golden or c2 or c3}" > gpurun_out/${TAG:-embpf}_tests.txt 2>&1 && \
run prof_base timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG:-embpf}_base -o run -- python3 bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/${TAG:-embpf}_base.log 2>&1 && \
PMG_LIB_PATH=$V run prof_var timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG:-embpf}_var -o run -- python3 bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/${TAG:-embpf}_var.log 2>&1 && \
PMG_LIB_PATH=$V run bench_var timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/${TAG:-embpf}_bench_var.json 2> gpurun_out/${TAG:-embpf}_bench_var.err && \
run bench_base timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/${TAG:-embpf}_bench_base.json 2> gpurun_out/${TAG:-embpf}_bench_base.err
