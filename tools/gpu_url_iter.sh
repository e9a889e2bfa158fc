# URL iteration loop on the GPU: parity tests, per-section clocks, bench (each step time-limited)
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_url_random.py tests/test_url_kats.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_url.log 2>&1 || { echo "url tests failed"; tail -40 gpurun_out/pytest_url.log; exit 1; }
tail -2 gpurun_out/pytest_url.log
timeout -k 10 200 python -u tools/url_clocks.py 10000000 > gpurun_out/url_clocks.log 2>&1 || { echo "clocks failed"; tail -20 gpurun_out/url_clocks.log; exit 1; }
grep clocks gpurun_out/url_clocks.log
timeout -k 10 300 python bench.py --workload ${1:-url} --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_iter.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_iter.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"kernel_ms_each": {[^}]*}' gpurun_out/bench_iter.log
