# full GPU suite, owner bench, C4 bench (no CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" gpurun_out/pytest_gpu.log | head -20; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 600 python -u bench.py --workload owner --steps 10 --warmup 3 > gpurun_out/r2_bench_owner.log 2>&1 || { echo "bench owner failed"; tail -30 gpurun_out/r2_bench_owner.log; exit 1; }
grep '"metric"' gpurun_out/r2_bench_owner.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_each'], d['config']['records'])"
timeout -k 10 600 python -u bench.py --workload fused --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2_bench_fused.log 2>&1 || { echo "bench fused failed"; tail -30 gpurun_out/r2_bench_fused.log; exit 1; }
grep '"metric"' gpurun_out/r2_bench_fused.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_each'], d.get('parity'))"
exit $rc
