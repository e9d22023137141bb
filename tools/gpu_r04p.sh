#!/bin/bash
# round 4 p: warm-up length x boundary tolerance sweep at C3 (driver window)
set -o pipefail
mkdir -p gpurun_out/r04p
export TMPDIR=/tmp
for cfg in "48 3e-6" "32 3e-6" "32 6e-6" "24 6e-6" "24 1e-5" "16 1e-5"; do
  set -- $cfg
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 --warm-steps $1 --scan-tol $2 \
    > gpurun_out/r04p/w$1_t$2.json 2> gpurun_out/r04p/w$1_t$2.err || exit 1
done
