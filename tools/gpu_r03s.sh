#!/bin/bash
# Round-3 session s: C5 batched-restart A/B, round-2 tree (exp/r02tree, built at a21660e) vs HEAD,
# each under a rocprofv3 kernel trace so per-launch relax/repair durations can be compared.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$PWD
cd "$R/exp/r02tree" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r03s_old" -o run --output-format csv -- \
  python3 -u bench.py --restarts 8 --no-cpu-baseline --no-api-fit > "$R/gpurun_out/r03s_old.json" 2> "$R/gpurun_out/r03s_old.err" &&
cd "$R" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r03s_new" -o run --output-format csv -- \
  python3 -u bench.py --restarts 8 --no-cpu-baseline --no-api-fit > "$R/gpurun_out/r03s_new.json" 2> "$R/gpurun_out/r03s_new.err"
