#!/bin/bash
# owner_fold per-phase clocks (diagnostic build _dg, OSE_OWNER_CLOCKS)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export OSE_SKIP_BUILD=1
OUT=$R/gpurun_out/r4l; mkdir -p $OUT
for w in owner sampling_wide; do
  OSE_LIB_VARIANT=_dg OSE_OWNER_CLOCKS=1 timeout -k 10 300 python -u bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $OUT/clk_$w.log 2>&1 || { tail -30 $OUT/clk_$w.log; exit 1; }
  echo "$w: $(grep "owner_fold clocks" $OUT/clk_$w.log | tail -1) $(grep -o "\"kernel_ms_each\": {[^}]*}" $OUT/clk_$w.log)"
done
