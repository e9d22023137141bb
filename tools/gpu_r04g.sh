#!/bin/bash
# round 4 g: full GPU suite at HEAD
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread > gpurun_out/r04g_tests.txt 2>&1
echo "suite rc=$?" >> gpurun_out/r04g_tests.txt
