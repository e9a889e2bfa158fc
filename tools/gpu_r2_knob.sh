#!/bin/bash
# grid sweep of the URL copy kernel on C4 (bench with env knobs)
set -o pipefail
mkdir -p gpurun_out/knob
run() {
  timeout -k 10 300 env "$@" python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/knob/b.log 2>&1 || { tail -20 gpurun_out/knob/b.log; exit 1; }
  echo "$@ $(grep -o '"url_copy_kernel": [0-9.]*' gpurun_out/knob/b.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/knob/b.log)"
}
run OSE_COPY_GRID=16384
run OSE_COPY_GRID=32768
run OSE_COPY_GRID=65536
run OSE_COPY_GRID=196000
