set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probe_scan_phases.py 8 quick > gpurun_out/r05_pv_base.txt 2>&1 || exit 1
for v in nt pf8 bpf4 sc1; do
  PMG_LIB_PATH=exp/$v/libpmg_hip.so timeout -k 10 200 python -u tools/probe_scan_phases.py 8 quick > gpurun_out/r05_pv_$v.txt 2>&1 || exit 1
done
