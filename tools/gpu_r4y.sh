#!/bin/bash
# table self-pointer for spilled routes: chunk/exchange/sampling suites, then
# the one-stream node8 kernel stats and the sampling line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export OSE_SKIP_BUILD=1
OUT=$R/gpurun_out/r4y; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_sampling_chunks.py tests/test_exchange.py tests/test_sampling_random.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/gpu_r4x.sh
