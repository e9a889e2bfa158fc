#!/bin/bash
# multi-chunk queue size / occupancy A/B, after the chunk tests on the default build
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r4ze
mkdir -p $OUT
cd $R
export OSE_SKIP_BUILD=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_sampling_chunks.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/gpu_ab.sh r4ze_ab _q64,_w4 sampling_wide
