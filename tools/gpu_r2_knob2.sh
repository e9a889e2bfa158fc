#!/bin/bash
# windows-per-wave sweep of trace_eval_kernel on C4 and C3
set -o pipefail
mkdir -p gpurun_out/knob
run() {
  wl=$1; shift
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/knob/b.log 2>&1 || { tail -20 gpurun_out/knob/b.log; exit 1; }
  echo "$wl $@ $(grep -o '"trace_eval_kernel": [0-9.]*' gpurun_out/knob/b.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/knob/b.log)"
}
for w in 8 16 24 32 64; do run fused OSE_WIN_PER_WAVE=$w; done
for w in 8 16 32; do run sampling OSE_WIN_PER_WAVE=$w; done
