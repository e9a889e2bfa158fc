#!/bin/bash
# dup bucket appends as atomic swaps (_dx): parity suite on the variant, A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export OSE_SKIP_BUILD=1
OUT=$R/gpurun_out/r4v; mkdir -p $OUT
OSE_LIB_VARIANT=_dx timeout -k 10 600 python -u -m pytest tests/test_sampling_random.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_dx.log 2>&1 || { tail -40 $OUT/pytest_dx.log; exit 1; }
tail -1 $OUT/pytest_dx.log
bash tools/gpu_ab.sh r4v_ab _dx sampling fused zipf
