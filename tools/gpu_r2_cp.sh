#!/bin/bash
# url_copy A/B on one box: one group per iteration at 8 waves/SIMD vs two groups at 5
mkdir -p gpurun_out/cp
for wl in fused zipf url; do
  for pr in 0 1 0 1; do
    OSE_COPY_PAIR=$pr timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/cp/${wl}_$pr.log 2>&1 || { tail -20 gpurun_out/cp/${wl}_$pr.log; exit 1; }
    echo "$wl pair=$pr $(grep -o '"url_copy_kernel": [0-9.]*' gpurun_out/cp/${wl}_$pr.log | head -1)"
  done
done
