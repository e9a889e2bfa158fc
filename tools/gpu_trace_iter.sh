set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sampling_kats.py tests/test_sampling_random.py tests/test_exchange.py tests/test_size.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_trace.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/pytest_trace.log | head; tail -40 gpurun_out/pytest_trace.log; exit 1; }
tail -2 gpurun_out/pytest_trace.log
timeout -k 10 300 python tools/ablate_trace.py 2>&1 | grep -v amdgpu.ids
