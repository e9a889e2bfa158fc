#!/bin/bash
# Round-3 bench lines of the other workloads (C2, C3, C5, owner side, the
# emulated 8-GPU step), groupbytrace, and the PMC traffic of C2 and C3.
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
OUT=gpurun_out/r3m
mkdir -p $OUT
for wl in url sampling zipf owner; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 20 --warmup 5 > $OUT/bench_$wl.log 2>&1 || { tail -20 $OUT/bench_$wl.log; exit 1; }
  echo "$wl $(grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"parity_vs_oracle": [a-z]*' $OUT/bench_$wl.log | tr '\n' ' ')"
done
timeout -k 10 400 python -u bench.py --workload node8 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_node8.log 2>&1 || { tail -20 $OUT/bench_node8.log; exit 1; }
echo "node8 $(grep -o '"projected_ms_per_gpu_step": [0-9.]*' $OUT/bench_node8.log)"
timeout -k 10 300 python -u tools/gbt_bench.py --out $OUT/gbt.json > $OUT/gbt.log 2>&1 || { tail -20 $OUT/gbt.log; exit 1; }
tail -3 $OUT/gbt.log
for wl in url sampling; do bash tools/pmc_traffic.sh $wl || exit 1; done
