# Round measurement: full GPU suite, then per workload a bench line (with the
# CPU baseline), rocprofv3 kernel stats and PMC HBM traffic.  Every step is
# time-limited; the script stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit 1
for wl in ${@:-fused url sampling zipf}; do
  bash tools/pmc_traffic.sh $wl || exit 1
done
python3 - <<'PY' || exit 1
import glob, json
d = {}
for f in sorted(glob.glob("gpurun_out/pmc_traffic_*.json")):
    for k, v in json.load(open(f)).items():
        d.setdefault(k, {}).update(v)
json.dump(d, open("gpurun_out/pmc_traffic.json", "w"), indent=1)
PY
for wl in ${@:-fused url sampling zipf}; do
  bash tools/gpu_bench_tj.sh $wl || exit 1
done
