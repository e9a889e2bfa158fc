# bench (PMC traffic from profiles/pmc_traffic.json) + rocprof kernel stats
# for the given workloads; each step time-limited, stop at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
for WL in ${@:-sampling zipf}; do
  timeout -k 10 400 python bench.py --workload $WL --steps 20 --warmup 5 > gpurun_out/bench_$WL.log 2>&1 || { echo "bench $WL failed"; tail -30 gpurun_out/bench_$WL.log; exit 1; }
  (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$WL -o $WL --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $WL --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_$WL.log 2>&1) || { echo "rocprof $WL failed"; tail -30 gpurun_out/prof_$WL.log; exit 1; }
done
