#!/bin/bash
# trace_eval with the service ids one step ahead (_tp, OSE_TE_PIPE=1): parity
# suites on the variant, then the A/B against the default build
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export OSE_SKIP_BUILD=1
OUT=$R/gpurun_out/r4q; mkdir -p $OUT
OSE_LIB_VARIANT=_tp timeout -k 10 600 python -u -m pytest tests/test_sampling_random.py tests/test_sampling_kats.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_tp.log 2>&1 || { tail -40 $OUT/pytest_tp.log; exit 1; }
tail -1 $OUT/pytest_tp.log
bash tools/gpu_ab.sh r4q_ab _tp sampling fused zipf
