# C5 / C3 / C2 bench lines with full-size parity, PMC HBM traffic per workload,
# kernel stats of C4 and of the owner-side workload
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
for wl in zipf sampling url; do
  echo "bench $wl"
  timeout -k 10 500 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2_bench_$wl.log 2>&1 || { echo "bench $wl failed"; tail -30 gpurun_out/r2_bench_$wl.log; exit 1; }
  grep '"metric"' gpurun_out/r2_bench_$wl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms_each'], d.get('parity'))"
done
for wl in fused sampling zipf url owner; do
  echo "pmc $wl"
  bash tools/pmc_traffic.sh $wl || exit 1
done
cd /tmp && export TMPDIR=/tmp
for wl in fused owner; do
  echo "kernel stats $wl"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$wl -o $wl -- python3 $GRAFT_REPO_ROOT/bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/gpurun_out/prof_$wl.log 2>&1 || { echo "rocprof $wl failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_$wl.log; exit 1; }
done
echo done
