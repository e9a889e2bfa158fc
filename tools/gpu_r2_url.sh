# URL parity tests, C4 bench (no CPU baseline), URL clocks
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_url_random.py tests/test_url_kats.py tests/test_size.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_url.log 2>&1 || { echo "url tests failed"; tail -30 gpurun_out/pytest_url.log; exit 1; }
tail -2 gpurun_out/pytest_url.log
timeout -k 10 600 python -u bench.py --workload fused --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2_bench_fused.log 2>&1 || { echo "bench fused failed"; tail -30 gpurun_out/r2_bench_fused.log; exit 1; }
grep '"metric"' gpurun_out/r2_bench_fused.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_each'], d.get('parity'))"
timeout -k 10 300 python -u tools/url_clocks.py 10000000 8 > gpurun_out/url_clocks.log 2>&1 || { echo "clocks failed"; tail -20 gpurun_out/url_clocks.log; exit 1; }
grep -v amdgpu.ids gpurun_out/url_clocks.log | head -3
