#!/bin/bash
# round-5 second evidence pass: default and driver-window bench lines, then the k_adam PMC
# passes on the shipped body (tools/gpu_adam_pmc.sh, OUT=r05i)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/r05b_default.json 2> gpurun_out/r05b_default.err && \
timeout -k 10 600 python -u bench.py --warmup 5 --steps 20 > gpurun_out/r05b_window.json 2> gpurun_out/r05b_window.err && \
OUT=r05i bash tools/gpu_adam_pmc.sh
