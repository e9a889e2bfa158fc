#!/bin/bash
# OTLP ingest with ScopeSpans walked on the GPU: OTLP/router/gbt tests, then the ingest-to-export bench
set -o pipefail
mkdir -p gpurun_out/o2
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_otlp.py tests/test_router_encode.py tests/test_groupbytrace.py > gpurun_out/o2/tests.log 2>&1
rc=$?
tail -3 gpurun_out/o2/tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/o2/tests.log | head -30; exit $rc; fi
timeout -k 10 500 python -u tools/otlp_bench.py --spans 10000000 --reps 4 --out gpurun_out/o2/otlp.json > gpurun_out/o2/otlp.log 2>&1 || { tail -30 gpurun_out/o2/otlp.log; exit 1; }
tail -1 gpurun_out/o2/otlp.log | cut -c1-1500
