R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4 -o run -- python3 $R/bench.py --shard time --config c4 --steps 3 --warmup 1 > $R/gpurun_out/prof_c4.log 2>&1
rc=$?; echo "prof rc=$rc"; head -20 $R/gpurun_out/prof_c4/run_kernel_stats.csv | cut -d, -f1-4
exit $rc
