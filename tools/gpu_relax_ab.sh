# relaxation-kernel A/B on the first iterations of a fresh C3 fit (tools/diag_iter1.py):
# the tree library and the exp/ variants in VARS, twice, interleaved
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for v in tree $VARS; do
  if [ $v = tree ]; then L=""; else L="PMG_LIB_PATH=exp/$v/libpmg_hip.so"; fi
  env $L timeout -k 10 120 python -u tools/diag_iter1.py --iters 2 --warms 48 > gpurun_out/rab_${v}_$rep.txt 2>&1 || exit 1
done
done
