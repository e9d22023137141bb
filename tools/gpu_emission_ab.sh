#!/bin/bash
# k_emission_lstat (default, 64 rows per wave), its 32-row form (exp/lsmr1) and k_emission_yreg (PMG_EMISSION_PIPE=2): emission parity tests,
# then kernel-trace durations of 55 back-to-back C3 calls each, twice
set -o pipefail
O=gpurun_out/r06ls
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "emission" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || exit 1
for rep in 1 2; do
  for v in lstat lsmr1 yreg; do
    unset PMG_EMISSION_PIPE PMG_LIB_PATH
    if [ $v = yreg ]; then export PMG_EMISSION_PIPE=2; fi
    if [ $v = lsmr1 ]; then export PMG_LIB_PATH=exp/lsmr1/libpmg_hip.so; fi
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_$rep -o run -- python3 tools/emission_bench.py > $O/${v}_$rep.log 2>&1 || exit 1
  done
done
