# GPU iteration for the SAMPLE stage: KATs + parity (each step time-limited)
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_sampling_kats.py tests/test_sampling_random.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_sampling.log 2>&1 || { echo "pytest sampling failed"; tail -60 gpurun_out/pytest_sampling.log; exit 1; }
tail -5 gpurun_out/pytest_sampling.log
