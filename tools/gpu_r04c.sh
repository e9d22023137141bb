#!/bin/bash
# round 4 c: planes statistics after the waterfall fix: focused tests, bench, kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "suffstats or planes or fit_em or adam_c3 or golden" > gpurun_out/r04c_tests.txt 2>&1
echo "tests rc=$?" >> gpurun_out/r04c_tests.txt
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 650 --timeout-method thread \
  tests/test_gpu_configs.py::test_c4_time_sharded_vs_single tests/test_gpu_timeshard.py > gpurun_out/r04c_c4.txt 2>&1
echo "c4 rc=$?" >> gpurun_out/r04c_c4.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04c_bench.json 2> gpurun_out/r04c_bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04c -o run -- python3 bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04c_prof.log 2>&1
timeout -k 10 300 python -u tools/api_fit_profile.py > gpurun_out/r04c_api_profile.json 2> gpurun_out/r04c_api_profile.err
timeout -k 10 200 python -u tools/adam_prof.py > gpurun_out/r04c_adamprof.txt 2>&1
