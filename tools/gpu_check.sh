# GPU round check: parity tests, bench, rocprofv3 kernel stats (run via gpurun from the repo root)
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu --timeout 400 > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
echo "bench ok"; tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1
echo "prof rc=$?"
