# bench + rocprofv3 kernel stats only (run via gpurun from the repo root)
TAG=${1:-run}
CFG=${2:-c3}
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --config $CFG --steps 19 --warmup 1 --no-cpu-baseline --no-api-fit > $R/gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 $R/gpurun_out/prof_$TAG.log | cut -c1-300
exit $rc
