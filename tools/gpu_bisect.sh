#!/bin/bash
# which variant of the library passes a set of GPU tests (each run time-limited;
# stops at a fault or time-out)
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out/bisect
for v in "$@"; do
  OSE_LIB_VARIANT=$v timeout -k 10 240 python -u -m pytest tests/test_concurrency.py tests/test_url_random.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/bisect/v$v.log 2>&1
  rc=$?
  echo "variant '$v': rc $rc: $(tail -1 gpurun_out/bisect/v$v.log)"
  grep -E "^FAILED" gpurun_out/bisect/v$v.log | head -5
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  if grep -q "illegal memory\|HIP error" gpurun_out/bisect/v$v.log; then exit 3; fi
done
