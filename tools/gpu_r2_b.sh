# GPU suite, then the C4 bench and the owner-side bench (each step time-limited).
# A pytest run with failing tests (rc 1) still lets the benches run; any other
# non-zero status (timeout, abort, fault) ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 600 python -u bench.py --workload fused --steps 20 --warmup 5 > gpurun_out/r2_bench_fused.log 2>&1 || { echo "bench fused failed"; tail -30 gpurun_out/r2_bench_fused.log; exit 1; }
grep '"metric"' gpurun_out/r2_bench_fused.log
timeout -k 10 600 python -u bench.py --workload owner --steps 10 --warmup 3 > gpurun_out/r2_bench_owner.log 2>&1 || { echo "bench owner failed"; tail -30 gpurun_out/r2_bench_owner.log; exit 1; }
grep '"metric"' gpurun_out/r2_bench_owner.log
exit $rc
