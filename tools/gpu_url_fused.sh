# URL parity tests, then C2 and C4 timings
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_url_random.py tests/test_url_kats.py tests/test_size.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_url.log 2>&1 || { echo "url tests failed"; tail -40 gpurun_out/pytest_url.log; exit 1; }
tail -1 gpurun_out/pytest_url.log
for wl in url fused; do
  timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_uf.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_uf.log; exit 1; }
  echo "$wl $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_uf.log) $(grep -o '"url_plan_kernel": [0-9.]*' gpurun_out/bench_uf.log)"
done
