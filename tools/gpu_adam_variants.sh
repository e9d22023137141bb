#!/bin/bash
# Adam body time per experiment build (exp/adam_*), then the Adam / EM parity tests on each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  PMG_LIB_PATH=exp/$v/libpmg_hip.so timeout -k 10 150 python -u tools/adam_prof.py 512 100000 512 300 \
    > gpurun_out/adamprof_$v.txt 2>&1 || exit 1
done
for v in "$@"; do
  PMG_LIB_PATH=exp/$v/libpmg_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
    -k "adam or fit_em or stop_rule" --timeout 120 --timeout-method thread > gpurun_out/adamtest_$v.txt 2>&1 || exit 1
done
