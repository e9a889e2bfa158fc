# concurrency + drop-in timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_concurrency.py tests/test_abi.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_conc.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|^ERROR|Error" gpurun_out/pytest_conc.log | head -20; tail -30 gpurun_out/pytest_conc.log; exit 1; }
tail -2 gpurun_out/pytest_conc.log
timeout -k 10 500 python -u tools/dropin_bench.py --out gpurun_out/r2_dropin.json 2>&1 | tee gpurun_out/r2_dropin.log
echo done
