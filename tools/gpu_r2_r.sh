#!/bin/bash
# round 2: ScopeSpans walked on the GPU: OTLP tests, then the ingest bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_otlp.py tests/test_router_encode.py tests/test_groupbytrace.py -m gpu > gpurun_out/r2r_tests.log 2>&1 || { tail -60 gpurun_out/r2r_tests.log; exit 1; }
tail -3 gpurun_out/r2r_tests.log
timeout -k 10 400 python -u tools/otlp_bench.py --spans 10000000 --reps 4 --out gpurun_out/r2r_otlp.json > gpurun_out/r2r_otlp.log 2>&1 || { tail -30 gpurun_out/r2r_otlp.log; exit 1; }
tail -1 gpurun_out/r2r_otlp.log
