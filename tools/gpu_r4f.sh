#!/bin/bash
# 5 waves per SIMD for url_plan_kernel (2 KiB stage, <= 96 VGPRs): URL GPU
# tests on the variant, then the A/B on C4 and C2
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export OSE_SKIP_BUILD=1
OUT=$R/gpurun_out/r4f; mkdir -p $OUT
OSE_LIB_VARIANT=_w5 timeout -k 10 600 python -u -m pytest tests/test_url_random.py tests/test_url_kats.py tests/test_url_refs.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_w5.log 2>&1 || { tail -30 $OUT/pytest_w5.log; exit 1; }
tail -1 $OUT/pytest_w5.log
bash tools/gpu_ab.sh r4f_w5 _w5 fused url
