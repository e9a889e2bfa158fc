#!/bin/bash
# bench lines for C3, C5 and the owner side with the current kernels
set -o pipefail
mkdir -p gpurun_out/b2
for wl in sampling zipf owner; do
  st=20; wu=5; if [ $wl = owner ]; then st=10; wu=3; fi
  timeout -k 10 500 python -u bench.py --workload $wl --steps $st --warmup $wu > gpurun_out/b2/bench_$wl.log 2>&1 || { tail -30 gpurun_out/b2/bench_$wl.log; exit 1; }
  echo "== $wl"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/b2/bench_$wl.log; grep -o '"frac": [0-9.]*' gpurun_out/b2/bench_$wl.log; grep -o '"parity_vs_oracle": [a-z]*' gpurun_out/b2/bench_$wl.log
done
