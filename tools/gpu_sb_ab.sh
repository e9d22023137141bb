set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probe_scan_phases.py 8 quick > gpurun_out/sb_probe_tree.txt 2>&1 || exit 1
PMG_LIB_PATH=exp/base/libpmg_hip.so timeout -k 10 200 python -u tools/probe_scan_phases.py 8 quick > gpurun_out/sb_probe_base.txt 2>&1 || exit 1
VARS="base" TAG=sb bash tools/gpu_bench_ab.sh
