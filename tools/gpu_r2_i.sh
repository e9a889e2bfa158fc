# sampling / exchange parity after the dup-flag change, owner + C3 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sampling_random.py tests/test_exchange.py tests/test_sampling_kats.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_samp.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|^ERROR|Error" gpurun_out/pytest_samp.log | head -20; tail -30 gpurun_out/pytest_samp.log; exit 1; }
tail -2 gpurun_out/pytest_samp.log
for wl in owner sampling; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r2_bench_$wl.log 2>&1 || { echo "bench $wl failed"; tail -30 gpurun_out/r2_bench_$wl.log; exit 1; }
  grep '"metric"' gpurun_out/r2_bench_$wl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_each'], d.get('parity'))"
done
echo done
