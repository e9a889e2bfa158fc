# OTLP ingest on the GPU + the suites the columniser refactor touches
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_otlp.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_otlp.log 2>&1 || { echo "otlp tests failed"; grep -E "^FAILED|^ERROR|Error|assert" gpurun_out/pytest_otlp.log | head -30; tail -40 gpurun_out/pytest_otlp.log; exit 1; }
tail -2 gpurun_out/pytest_otlp.log
timeout -k 10 600 python -u -m pytest tests/test_size.py tests/test_span_attribute.py tests/test_concurrency.py tests/test_url_kats.py tests/test_sampling_kats.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_misc.log 2>&1 || { echo "misc tests failed"; grep -E "^FAILED|^ERROR" gpurun_out/pytest_misc.log | head; tail -30 gpurun_out/pytest_misc.log; exit 1; }
tail -2 gpurun_out/pytest_misc.log
echo done
