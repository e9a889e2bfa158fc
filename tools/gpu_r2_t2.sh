#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_url_random.py > gpurun_out/t2_tests.log 2>&1
rc=$?
tail -12 gpurun_out/t2_tests.log
exit $rc
