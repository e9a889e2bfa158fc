#!/bin/bash
# size_span_kernel grid cap sweep at C4's 100M spans
mkdir -p gpurun_out/sg
for gsz in 1024 2048 4096 8192 1024 4096; do
  OSE_SIZE_GRID=$gsz timeout -k 10 300 python -u bench.py --workload fused --steps 10 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/sg/fused_$gsz.log 2>&1 || { tail -20 gpurun_out/sg/fused_$gsz.log; exit 1; }
  echo "fused grid=$gsz $(grep -o '"size_span_kernel": [0-9.]*' gpurun_out/sg/fused_$gsz.log | head -1)"
done
