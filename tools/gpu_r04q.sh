#!/bin/bash
# round 4 q: n_latent_bin > 1024 through the dense scans (JD = 8)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_dense.py > gpurun_out/r04q_tests.txt 2>&1
echo "rc=$?" >> gpurun_out/r04q_tests.txt
