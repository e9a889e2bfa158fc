# bench + rocprof kernel stats for one workload (each step time-limited)
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
WL=${1:-url}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload $WL --steps 20 --warmup 5 --traffic-json gpurun_out/pmc_traffic.json > gpurun_out/bench_$WL.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_$WL.log; exit 1; }
grep '"metric"' gpurun_out/bench_$WL.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$WL -o $WL --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $WL --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_$WL.log 2>&1 || { echo "rocprof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_$WL.log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/gpurun_out/prof_$WL -name "*kernel_stats.csv" | head -1)
head -12 "$f"
