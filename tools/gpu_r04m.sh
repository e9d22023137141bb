#!/bin/bash
# round 4 m: warm-up band cut (warm_band): bench first, then the full GPU suite
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r04m_steps.txt; return $rc; }
: > gpurun_out/r04m_steps.txt
run bench timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04m_bench.json 2> gpurun_out/r04m_bench.err && \
run suite timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r04m_tests.txt 2>&1
