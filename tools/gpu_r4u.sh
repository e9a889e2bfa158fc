#!/bin/bash
# size spans pass: plain stores for wave-interior scopes (_sp) — parity
# suites on the variant, the fused line with parity, then the A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export OSE_SKIP_BUILD=1
OUT=$R/gpurun_out/r4u; mkdir -p $OUT
OSE_LIB_VARIANT=_sp timeout -k 10 600 python -u -m pytest tests/test_size.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_sp.log 2>&1 || { tail -40 $OUT/pytest_sp.log; exit 1; }
tail -1 $OUT/pytest_sp.log
OSE_LIB_VARIANT=_sp timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_fused_sp.log 2>&1 || { tail -30 $OUT/bench_fused_sp.log; exit 1; }
grep -o '"parity": {[^}]*}' $OUT/bench_fused_sp.log
bash tools/gpu_ab.sh r4u_ab _sp fused
