#!/bin/bash
# Round-2 final measurement: C3 bench (+ CPU baseline, public-API fit), its rocprofv3 kernel
# trace, the PMC passes, the C4 one-GPU time-shard bench (first-iteration scans), C5 batched
# restarts.  Every step has its own time limit; the chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02h}
timeout -k 10 400 python -u bench.py > gpurun_out/bench_${TAG}_c3.json 2> gpurun_out/bench_${TAG}_c3.err &&
bash tools/gpu_prof.sh ${TAG}_c3 c3 &&
bash tools/gpu_pmc.sh pmc_${TAG} c3 &&
timeout -k 10 300 python -u bench.py --restarts 8 --no-cpu-baseline > gpurun_out/bench_${TAG}_c5.json 2> gpurun_out/bench_${TAG}_c5.err &&
timeout -k 10 500 python -u bench.py --config c4 --shard time --warmup 1 --steps 3 > gpurun_out/bench_${TAG}_c4.json 2> gpurun_out/bench_${TAG}_c4.err
