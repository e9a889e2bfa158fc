#!/bin/bash
# span_attribute rules past 64 (attr_match words), chunked exchange, the
# whole GPU suite, smoke, the C4 line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export OSE_SKIP_BUILD=1
OUT=$R/gpurun_out/r4g; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_span_attribute.py tests/test_sampling_chunks.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_attr.log 2>&1 || { tail -40 $OUT/pytest_attr.log; exit 1; }
tail -1 $OUT/pytest_attr.log
bash tools/gpu_check.sh r4g fused
