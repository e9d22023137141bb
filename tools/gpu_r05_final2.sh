#!/bin/bash
# round-5 closing evidence after the tuning tiles: full GPU suite, then tools/gpu_r05_final.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r05g_tests.txt 2>&1 && \
bash tools/gpu_r05_final.sh
