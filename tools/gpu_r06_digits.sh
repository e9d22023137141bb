#!/bin/bash
# closing suite + smoke on the tree library, then the 4-digit emission variant (exp/dig4,
# PMG_EMISSION_DIGITS=4) against the tree in the driver window, interleaved twice
set -o pipefail
O=${O:-gpurun_out/r06fin}
mkdir -p $O
export TMPDIR=/tmp
O=$O bash tools/gpu_r06_suite.sh && \
VARS=dig4 TAG=r06fin/ab bash tools/gpu_bench_ab.sh
