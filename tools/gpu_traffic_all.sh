# bench line for one workload, then PMC HBM traffic for every workload (each step time-limited)
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload ${1:-zipf} --steps 20 --warmup 5 > gpurun_out/bench_${1:-zipf}.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_${1:-zipf}.log; exit 1; }
grep '"metric"' gpurun_out/bench_${1:-zipf}.log
for wl in url sampling zipf fused; do
  bash tools/pmc_traffic.sh $wl || exit 1
done
