#!/bin/bash
# windows per wave of trace_eval_kernel after the lean instance: C3 and C4
mkdir -p gpurun_out/wpw
for wl in sampling fused; do
  for w in 8 16 32 64; do
    OSE_WIN_PER_WAVE=$w timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/wpw/${wl}_$w.log 2>&1 || { tail -20 gpurun_out/wpw/${wl}_$w.log; exit 1; }
    echo "$wl wpw=$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/wpw/${wl}_$w.log) $(grep -o '"trace_eval_kernel": [0-9.]*' gpurun_out/wpw/${wl}_$w.log | head -1)"
  done
done
