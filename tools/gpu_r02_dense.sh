#!/bin/bash
# Dense log-domain scans + parity fixes: the new tests and the suites they touch.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_timeshard.py tests/test_gpu_model_selection.py \
    "tests/test_gpu_parity.py::test_latent_only_decode_vs_oracle" "tests/test_gpu_parity.py::test_latent_only_fit_em_one_iteration_vs_oracle" \
    -v --timeout 300 --timeout-method thread > gpurun_out/t_dense.log 2>&1
