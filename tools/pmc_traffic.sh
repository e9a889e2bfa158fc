# HBM traffic of the bench workload per launch (MI355X_MICROARCH.md "HBM [CDNA4]"):
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (kernel-trace only); the
# summariser doubles FETCH_SIZE (gfx950 tallies 128-B read requests at 64 B).
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
WL=${1:-url}
mkdir -p gpurun_out/traffic_$WL
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/traffic_$WL/$ctr -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/gpurun_out/traffic_$WL/$ctr.log 2>&1 || { echo "pmc $ctr failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/traffic_$WL/$ctr.log; exit 1; }
done
python3 $GRAFT_REPO_ROOT/tools/pmc_traffic.py $WL $GRAFT_REPO_ROOT/gpurun_out/traffic_$WL $GRAFT_REPO_ROOT/gpurun_out/pmc_traffic_$WL.json
