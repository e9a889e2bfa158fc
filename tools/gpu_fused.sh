set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_exchange.py tests/test_size.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_x.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_x.log; exit 1; }
tail -3 gpurun_out/pytest_x.log
bash tools/gpu_bench.sh fused
