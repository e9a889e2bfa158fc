#!/bin/bash
# localize a host heap corruption seen at exit of a combined run
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
timeout -k 10 300 python -u -X faulthandler -m pytest -x -q --timeout 150 --timeout-method thread tests/test_otlp.py tests/test_router_encode.py tests/test_groupbytrace.py -m gpu > gpurun_out/r2s_all.log 2>&1
rc=$?
echo "rc=$rc"; tail -60 gpurun_out/r2s_all.log
exit 0
