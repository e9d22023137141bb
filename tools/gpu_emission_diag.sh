#!/bin/bash
# kernel-trace durations of the C3 emission for the tree and the timing-diagnostic variants
set -o pipefail
O=gpurun_out/r06ed2
mkdir -p $O
export TMPDIR=/tmp
for v in tree ${VARS:-ediag1 ediag2}; do
  if [ $v = tree ]; then unset PMG_LIB_PATH; else export PMG_LIB_PATH=exp/$v/libpmg_hip.so; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 tools/emission_bench.py > $O/$v.log 2>&1 || exit 1
done
