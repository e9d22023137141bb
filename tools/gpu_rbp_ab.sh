# emission block-maxima store runs: parity with the variant, then interleaved window benches
# of the tree library and the exp/ variants in VARS
set -o pipefail
mkdir -p gpurun_out
for v in $VARS; do
  PMG_LIB_PATH=exp/$v/libpmg_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "emission" > gpurun_out/rbp_tests_$v.txt 2>&1 || exit 1
done
for rep in 1 2 3; do
  for v in tree $VARS; do
    if [ $v = tree ]; then L=""; else L="PMG_LIB_PATH=exp/$v/libpmg_hip.so"; fi
    env $L timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-api-fit > gpurun_out/rbp_${v}_$rep.json 2>/dev/null || exit 1
  done
done
