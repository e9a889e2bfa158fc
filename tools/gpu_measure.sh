# bench + rocprof stats + PMC HBM traffic for the given workloads
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
for wl in "$@"; do
  bash tools/gpu_bench.sh $wl || exit 1
  bash tools/pmc_traffic.sh $wl || exit 1
done
