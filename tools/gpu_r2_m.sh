#!/bin/bash
# round 2: output side on the GPU (router + re-encode tests), OTLP bench with the encode leg
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_router_encode.py tests/test_otlp.py -m gpu > gpurun_out/r2n_tests.log 2>&1 || { tail -40 gpurun_out/r2n_tests.log; exit 1; }
tail -3 gpurun_out/r2n_tests.log
timeout -k 10 400 python -u tools/otlp_bench.py --spans 10000000 --reps 4 --out gpurun_out/r2n_otlp.json > gpurun_out/r2n_otlp.log 2>&1 || { tail -30 gpurun_out/r2n_otlp.log; exit 1; }
tail -2 gpurun_out/r2n_otlp.log
