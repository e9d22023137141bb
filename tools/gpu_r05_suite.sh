#!/bin/bash
# round-5 evidence, part 1: the whole GPU suite and smoke
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 700 --timeout-method thread -m gpu tests/ > gpurun_out/r05_gpu_tests.txt 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.txt 2>&1
