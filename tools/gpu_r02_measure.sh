#!/bin/bash
# Round-2 measurement: C3 bench (fresh fit, fp32 all-core CPU baseline, public-API fit),
# the rocprofv3 kernel trace of the same bench, and the PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02}
timeout -k 10 400 python -u bench.py > gpurun_out/bench_${TAG}_c3.json 2> gpurun_out/bench_${TAG}_c3.err &&
bash tools/gpu_prof.sh ${TAG}_c3 c3 &&
bash tools/gpu_pmc.sh pmc_${TAG} c3
