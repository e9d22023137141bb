#!/bin/bash
# round 4, first GPU pass: new parity tests (C3 Adam instance, C1 README fit, Adam timeout)
# on the hardware-transcendental softplus, then C3 benches: new Adam vs the round-3 OCML form
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
  "tests/test_gpu_parity.py::test_adam_vs_oracle" \
  tests/test_gpu_parity.py::test_adam_c3_full_loop_vs_f64_ensemble \
  tests/test_gpu_parity.py::test_fit_em_c1_readme_golden \
  tests/test_gpu_parity.py::test_fit_em_stop_rule_golden \
  tests/test_gpu_parity.py::test_fit_em_fixed_iterations_golden \
  tests/test_gpu_configs.py::test_c3_one_em_iteration_vs_oracle \
  tests/test_gpu_configs.py::test_c2_one_em_iteration_vs_oracle \
  tests/test_gpu_status.py > gpurun_out/r04a_tests.txt 2>&1
echo "tests rc=$?" >> gpurun_out/r04a_tests.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04a_bench_new.json 2> gpurun_out/r04a_bench_new.err && \
PMG_LIB_PATH=exp/spocml/libpmg_hip.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-fit --warmup 5 --steps 20 > gpurun_out/r04a_bench_ocml.json 2> gpurun_out/r04a_bench_ocml.err && \
timeout -k 10 600 python -u bench.py --no-cpu-baseline --decode > gpurun_out/r04a_bench_decode.json 2> gpurun_out/r04a_bench_decode.err
