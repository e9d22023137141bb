#!/bin/bash
# Round-2 relaxation check: cascade diagnostic, the scan parity tests and a C3 bench.
# Each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_cascade.py c3 6 > gpurun_out/diag_relax_c3.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "forward_backward or cascade or masked_latents_scan" > gpurun_out/t_scan.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1
