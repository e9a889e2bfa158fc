#!/bin/bash
# size records: size/OTLP GPU tests, C4 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_size.py tests/test_otlp.py tests/test_router_encode.py tests/test_groupbytrace.py tests/test_abi.py > gpurun_out/r2z_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r2z_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r2z_tests.log | head -30; exit $rc; fi
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2z_bench_fused.log 2>&1 || { tail -30 gpurun_out/r2z_bench_fused.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2z_bench_fused.log
grep -o '"kernel_ms_each": {[^}]*}' gpurun_out/r2z_bench_fused.log
grep -o '"parity": {[^}]*}' gpurun_out/r2z_bench_fused.log
