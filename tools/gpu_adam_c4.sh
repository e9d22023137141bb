# tiled-Adam parity + C4 time-shard profile (run via gpurun from the repo root)
TAG=${1:-a}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k adam -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_adam_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_adam_$TAG.log
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4_$TAG -o run -- python3 $R/bench.py --shard time --config c4 --steps 3 --warmup 1 > $R/gpurun_out/prof_c4_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; head -14 $R/gpurun_out/prof_c4_$TAG/run_kernel_stats.csv | cut -d, -f1-4
tail -1 $R/gpurun_out/prof_c4_$TAG.log | cut -c1-300
exit $rc
