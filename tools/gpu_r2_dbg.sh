#!/bin/bash
# which test leaves a HIP error in the runtime (conftest guard names it)
mkdir -p gpurun_out/dbg
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_otlp.py tests/test_url_kats.py tests/test_size.py > gpurun_out/dbg/guard.log 2>&1
rc=$?
echo "rc=$rc"; tail -3 gpurun_out/dbg/guard.log; grep -E "^(ERROR|FAILED)|left in the runtime" gpurun_out/dbg/guard.log | head -20
