#!/bin/bash
# round-6 closing bench lines on the final library (no PMC: the C3 kernels the PMC passes
# cover are unchanged since profiles/r06_pmc_c3.json): default and driver-window lines, the
# rocprofv3 kernel trace of the driver window, C5 restarts, C1, C2, C4 unsharded
set -o pipefail
O=${O:-gpurun_out/r06close}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > $O/default.json 2> $O/default.err && \
timeout -k 10 600 python -u bench.py --warmup 5 --steps 20 --decode > $O/window.json 2> $O/window.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > $O/prof.log 2>&1 && \
timeout -k 10 300 python -u bench.py --restarts 8 --no-cpu-baseline > $O/c5.json 2> $O/c5.err && \
timeout -k 10 300 python -u bench.py --config c1 --no-api-fit > $O/c1.json 2> $O/c1.err && \
timeout -k 10 300 python -u bench.py --config c2 --no-api-fit > $O/c2.json 2> $O/c2.err && \
timeout -k 10 500 python -u bench.py --config c4 --no-cpu-baseline --no-api-fit --warmup 2 --steps 5 > $O/c4.json 2> $O/c4.err
