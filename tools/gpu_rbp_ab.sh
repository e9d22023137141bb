set -o pipefail
mkdir -p gpurun_out
PMG_LIB_PATH=exp/rbp/libpmg_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "emission" > gpurun_out/rbp_tests.txt 2>&1 || exit 1
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-api-fit > gpurun_out/rbp_tree_$rep.json 2>/dev/null && \
  PMG_LIB_PATH=exp/rbp/libpmg_hip.so timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-api-fit > gpurun_out/rbp_var_$rep.json 2>/dev/null || exit 1
done
