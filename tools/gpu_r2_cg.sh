#!/bin/bash
# url_copy_kernel grid sweep on C4 and C2
mkdir -p gpurun_out/cg
for wl in fused url; do
  for gsz in 16384 32768 65536 131072; do
    OSE_COPY_GRID=$gsz timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/cg/${wl}_$gsz.log 2>&1 || { tail -20 gpurun_out/cg/${wl}_$gsz.log; exit 1; }
    echo "$wl grid=$gsz $(grep -o '"url_copy_kernel": [0-9.]*' gpurun_out/cg/${wl}_$gsz.log | head -1)"
  done
done
