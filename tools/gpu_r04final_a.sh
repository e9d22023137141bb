#!/bin/bash
# round 4 final (a): smoke, default bench (driver form), rocprof kernel trace/stats of the
# driver-window bench, PMC passes; each step bounded, chained with &&
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r04ja_steps.txt; return $rc; }
: > gpurun_out/r04ja_steps.txt
run smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04ja_smoke.txt 2>&1 && \
run bench_default timeout -k 10 600 python -u bench.py > gpurun_out/r04ja_bench_default.json 2> gpurun_out/r04ja_bench_default.err && \
run bench_window timeout -k 10 300 python -u bench.py --no-cpu-baseline --warmup 5 --steps 20 --decode > gpurun_out/r04ja_bench_window.json 2> gpurun_out/r04ja_bench_window.err && \
run prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04ja -o run -- python3 bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04ja_prof.log 2>&1 && \
if [ -n "$PMC" ]; then run pmc bash tools/gpu_pmc.sh r04gpmc c3; fi
