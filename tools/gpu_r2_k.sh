# OTLP ingest: GPU tests + timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_otlp.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_otlp.log 2>&1 || { echo "otlp tests failed"; grep -E "^FAILED|^ERROR|Error|assert" gpurun_out/pytest_otlp.log | head -30; tail -30 gpurun_out/pytest_otlp.log; exit 1; }
tail -2 gpurun_out/pytest_otlp.log
timeout -k 10 500 python -u tools/otlp_bench.py --spans 10000000 --out gpurun_out/r2_otlp.json 2>&1 | tee gpurun_out/r2_otlp.log
echo done
