#!/bin/bash
# Round-3: full GPU suite at HEAD, then the C3 bench and its rocprofv3 kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03a}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench_${TAG}_c3.json 2> gpurun_out/bench_${TAG}_c3.err &&
bash tools/gpu_prof.sh ${TAG}_c3 c3
