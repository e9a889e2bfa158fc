# long-run tuning: sampling parity, then zipf and C3 timings per hand-off distance
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sampling_random.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_samp.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_samp.log; exit 1; }
tail -1 gpurun_out/pytest_samp.log
for ls in ${@:-16}; do
  for wl in zipf sampling; do
    OSE_LONG_STEPS=$ls timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_l.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_l.log; exit 1; }
    echo "$ls $wl $(grep -o '"kernel_ms_each": {[^}]*}' gpurun_out/bench_l.log)"
  done
done
