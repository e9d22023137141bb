#!/bin/bash
# Adam table-exp variant: body time A/B (tools/adam_prof.py, C3, 300 fixed bodies, interleaved
# twice), a driver-window bench pair, then the Adam / stop-rule / C1-README / C2-multi tests
# on the variant library
set -o pipefail
O=gpurun_out/r06ad
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 200 python -u tools/adam_prof.py 512 100000 512 300 > $O/tree_$rep.txt 2>&1 || exit 1
  PMG_LIB_PATH=exp/adtab/libpmg_hip.so timeout -k 10 200 python -u tools/adam_prof.py 512 100000 512 300 > $O/adtab_$rep.txt 2>&1 || exit 1
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > $O/bench_tree.json 2>/dev/null || exit 1
PMG_LIB_PATH=exp/adtab/libpmg_hip.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > $O/bench_adtab.json 2>/dev/null || exit 1
PMG_LIB_PATH=exp/adtab/libpmg_hip.so timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_timeshard.py tests/test_gpu_restarts.py tests/test_gpu_configs.py tests/test_gpu_tuning.py \
  -k "adam or stop_rule or readme or neuron_sharded or c2_multi or c3_one_em or fit_em" > $O/tests_adtab.txt 2>&1
