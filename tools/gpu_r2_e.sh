# concurrency tests, drop-in timing, owner bench + its kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_concurrency.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_conc.log 2>&1 || { echo "concurrency tests failed"; tail -40 gpurun_out/pytest_conc.log; exit 1; }
tail -2 gpurun_out/pytest_conc.log
timeout -k 10 400 python -u tools/dropin_bench.py --out gpurun_out/r2_dropin.json > gpurun_out/r2_dropin.log 2>&1 || { echo "dropin failed"; tail -30 gpurun_out/r2_dropin.log; exit 1; }
tail -c 3000 gpurun_out/r2_dropin.log
timeout -k 10 300 python -u bench.py --workload owner --steps 10 --warmup 3 > gpurun_out/r2_bench_owner.log 2>&1 || { echo "bench owner failed"; tail -30 gpurun_out/r2_bench_owner.log; exit 1; }
grep '"metric"' gpurun_out/r2_bench_owner.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_each'], d['config']['records'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_owner -o owner -- python3 $GRAFT_REPO_ROOT/bench.py --workload owner --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_owner.log 2>&1 || { echo "rocprof owner failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_owner.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_owner -name "*kernel_stats.csv" | head -3
echo done
