set -o pipefail
mkdir -p gpurun_out
for v in tree a1 pf4 a1pf4 bpf2 bm all; do
  if [ $v = tree ]; then L=""; else L="PMG_LIB_PATH=exp/$v/libpmg_hip.so"; fi
  env $L timeout -k 10 120 python -u tools/diag_iter1.py --iters 2 --warms 48 > gpurun_out/rab_$v.txt 2>&1 || exit 1
done
