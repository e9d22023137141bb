#!/bin/bash
# full GPU suite, the first iterations of a fresh C3 fit, and the driver-window bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r05c_tests.txt 2>&1 && \
timeout -k 10 120 python -u tools/diag_iter1.py --iters 3 --warms 48 > gpurun_out/r05c_iter1.txt 2>&1 && \
timeout -k 10 600 python -u bench.py --warmup 5 --steps 20 > gpurun_out/r05c_window.json 2> gpurun_out/r05c_window.err
