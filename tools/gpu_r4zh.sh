#!/bin/bash
# sparse rule walk in the one-table lean trace_eval instances: A/B on C4 and
# C3, then the sampling suites on the variant build
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r4zh
mkdir -p $OUT
cd $R
export OSE_SKIP_BUILD=1
bash tools/gpu_ab.sh r4zh_ab _sw fused sampling || exit 1
OSE_LIB_VARIANT=_sw timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sampling_random.py tests/test_sampling_kats.py tests/test_exchange.py tests/test_sampling_chunks.py tests/test_span_attribute.py > $OUT/pytest_sw.log 2>&1 || { tail -40 $OUT/pytest_sw.log; exit 1; }
tail -1 $OUT/pytest_sw.log
