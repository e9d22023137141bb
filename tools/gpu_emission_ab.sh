#!/bin/bash
# the tree emission and experiment variants (VARS="a b": exp/NAME/libpmg_hip.so): the tree's emission parity tests,
# then kernel-trace durations of 55 back-to-back C3 calls each, twice
set -o pipefail
O=${O:-gpurun_out/r06ls}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "emission" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || exit 1
for rep in 1 2; do
  for v in tree ${VARS}; do
    unset PMG_LIB_PATH
    if [ $v != tree ]; then export PMG_LIB_PATH=exp/$v/libpmg_hip.so; fi
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_$rep -o run -- python3 tools/emission_bench.py > $O/${v}_$rep.log 2>&1 || exit 1
  done
done
