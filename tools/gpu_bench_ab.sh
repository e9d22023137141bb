#!/bin/bash
# driver-window bench of the tree library and of experiment variants, interleaved twice:
#   VARS="a b" TAG=x bash tools/gpu_bench_ab.sh   (variants from exp/NAME/libpmg_hip.so)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-ab}
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/${TAG}_base_$rep.json 2> gpurun_out/${TAG}_base_$rep.err || exit 1
  for v in $VARS; do
    PMG_LIB_PATH=exp/$v/libpmg_hip.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/${TAG}_${v}_$rep.json 2> gpurun_out/${TAG}_${v}_$rep.err || exit 1
  done
done
