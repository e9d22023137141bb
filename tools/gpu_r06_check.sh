set -o pipefail
mkdir -p gpurun_out/r06d
tools/gpu_chunk_ab.sh gpurun_out/r06d/ab "49,98 49,98 49,98" 1 > gpurun_out/r06d/ab.txt 2>&1 || exit 1
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06d/gpu_tests.txt 2>&1
