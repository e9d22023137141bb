set -o pipefail
mkdir -p gpurun_out/r06f
tools/gpu_chunk_ab.sh gpurun_out/r06f/ab "49,98 49,98 49,98" 1 > gpurun_out/r06f/ab.txt 2>&1 || exit 1
timeout -k 10 240 python -u tools/probe_scan_phases.py 8 quick > gpurun_out/r06f/probe.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_relax_settle.py tests/test_gpu_restarts.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06f/tests.txt 2>&1
