#!/bin/bash
# round 4, first GPU pass: new parity tests (C3 Adam instance, C1 README fit, Adam timeout),
# then a C3 bench with the decode leg
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
  "tests/test_gpu_parity.py::test_adam_vs_oracle" \
  tests/test_gpu_parity.py::test_adam_c3_full_loop_vs_f64_ensemble \
  tests/test_gpu_parity.py::test_fit_em_c1_readme_golden \
  tests/test_gpu_status.py > gpurun_out/r04a_tests.txt 2>&1 && \
timeout -k 10 600 python -u bench.py --no-cpu-baseline --decode > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err
