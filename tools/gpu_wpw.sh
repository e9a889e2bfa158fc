# windows-per-wave sweep of the trace kernel (C3, C5, C4)
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sampling_random.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_samp.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_samp.log; exit 1; }
tail -1 gpurun_out/pytest_samp.log
for w in ${@:-8}; do
  for wl in sampling zipf fused; do
    OSE_WIN_PER_WAVE=$w timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_w.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_w.log; exit 1; }
    echo "$w $wl $(grep -o '"trace_eval_kernel": [0-9.]*' gpurun_out/bench_w.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_w.log)"
  done
done
