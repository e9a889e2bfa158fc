#!/bin/bash
# round 2: groupbytrace store on the GPU
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_groupbytrace.py tests/test_otlp.py tests/test_router_encode.py tests/test_concurrency.py -m gpu > gpurun_out/r2o_tests.log 2>&1 || { tail -60 gpurun_out/r2o_tests.log; exit 1; }
tail -5 gpurun_out/r2o_tests.log
