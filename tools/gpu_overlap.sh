# fused parity tests, then the fused bench with and without the SAMPLE || TEMPLATE overlap
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_size.py tests/test_exchange.py tests/test_url_random.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ov.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_ov.log; exit 1; }
tail -1 gpurun_out/pytest_ov.log
for ov in 0 1; do
  if [ $ov = 0 ]; then export OSE_NO_OVERLAP=1; else unset OSE_NO_OVERLAP; fi
  timeout -k 10 300 python bench.py --workload fused --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_ov.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_ov.log; exit 1; }
  echo "overlap=$ov $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_ov.log)"
done
timeout -k 10 200 python tools/slowpath_time.py 12500000
