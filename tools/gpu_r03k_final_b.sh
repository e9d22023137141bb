#!/bin/bash
# Round-3 final (b, after the emission rewrite): rocprofv3 kernel stats of the C3 bench, then the PMC passes (one counter group per run).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_prof.sh r03kfinal c3 && bash tools/gpu_pmc.sh r03kpmc c3
