#!/bin/bash
# Adam body A/B: tools/adam_prof.py (C3, 300 fixed bodies) on the tree library and on the
# exp/NAME variants in VARS, interleaved twice; then the Adam oracle tests on the tree.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-adam}
for rep in 1 2; do
  timeout -k 10 200 python -u tools/adam_prof.py 512 100000 512 300 > gpurun_out/${TAG}_tree_$rep.txt 2>&1 || exit 1
  for v in $VARS; do
    PMG_LIB_PATH=exp/$v/libpmg_hip.so timeout -k 10 200 python -u tools/adam_prof.py 512 100000 512 300 > gpurun_out/${TAG}_${v}_$rep.txt 2>&1 || exit 1
  done
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_timeshard.py tests/test_gpu_restarts.py \
  -k "${SEL:-adam or stop_rule or readme or neuron_sharded}" > gpurun_out/${TAG}_tests.txt 2>&1
