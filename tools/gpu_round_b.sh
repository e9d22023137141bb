# PMC passes at C3 (counters only, one rocprofv3 run per pass), chunk sweep, C4 time-shard bench
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_pmc.sh pmcb c3 || exit 1
bash tools/chunk_sweep.sh || exit 1
timeout -k 10 400 python -u bench.py --shard time --config c4 --steps 5 --warmup 2 > gpurun_out/bench_c4_b.log 2>&1 || { echo "c4 failed"; tail -5 gpurun_out/bench_c4_b.log; exit 1; }
tail -1 gpurun_out/bench_c4_b.log | cut -c1-300
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4_b -o run -- python3 $R/bench.py --shard time --config c4 --steps 3 --warmup 1 > $R/gpurun_out/prof_c4_b.log 2>&1
echo "c4 prof rc=$?"
