#!/bin/bash
# round-6 closing evidence, part 1: the whole -m gpu suite and smoke() on one box
set -o pipefail
O=${O:-gpurun_out/r06z}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
