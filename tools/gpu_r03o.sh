#!/bin/bash
# Round-3 session o: Adam with one exp / one reciprocal per row slot (PMG_ADAM_FASTSP=1 build): parity + A/B bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PMG_LIB_PATH=exp/fastsp/libpmg_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread \
  -k "adam or em_ or golden or c3 or c5 or c2 or fit" > gpurun_out/r03o_tests.txt 2>&1
echo "tests rc=$?" >> gpurun_out/r03o_tests.txt
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r03o_bench_base.json 2> gpurun_out/r03o_bench_base.err &&
PMG_LIB_PATH=exp/fastsp/libpmg_hip.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r03o_bench_fastsp.json 2> gpurun_out/r03o_bench_fastsp.err &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r03o_bench_base2.json 2> gpurun_out/r03o_bench_base2.err &&
PMG_LIB_PATH=exp/fastsp/libpmg_hip.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r03o_bench_fastsp2.json 2> gpurun_out/r03o_bench_fastsp2.err
