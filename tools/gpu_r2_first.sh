# Round 2, first measurement: C4 at 100M spans on one GPU (bench + parity),
# the owner-side workload, kernel stats of the fused step.
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --workload fused --steps 20 --warmup 5 > gpurun_out/r2_bench_fused.log 2>&1 || { echo "bench fused failed"; tail -30 gpurun_out/r2_bench_fused.log; exit 1; }
grep '"metric"' gpurun_out/r2_bench_fused.log
timeout -k 10 600 python -u bench.py --workload owner --steps 10 --warmup 3 > gpurun_out/r2_bench_owner.log 2>&1 || { echo "bench owner failed"; tail -30 gpurun_out/r2_bench_owner.log; exit 1; }
grep '"metric"' gpurun_out/r2_bench_owner.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2_prof_fused -o fused --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload fused --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/gpurun_out/r2_prof_fused.log 2>&1 || { echo "rocprof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/r2_prof_fused.log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/gpurun_out/r2_prof_fused -name "*kernel_stats.csv" | head -1)
head -14 "$f"
