#!/bin/bash
# lane-per-run trace kernel: sampling/exchange/attr GPU tests, then C3, C4, C5, owner benches
set -o pipefail
mkdir -p gpurun_out/l2
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_sampling_random.py tests/test_sampling_kats.py tests/test_exchange.py tests/test_span_attribute.py tests/test_groupbytrace.py tests/test_concurrency.py > gpurun_out/l2/tests.log 2>&1
rc=$?
tail -3 gpurun_out/l2/tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/l2/tests.log | head -30; exit $rc; fi
for wl in sampling fused zipf owner; do
  st=20; wu=5; if [ $wl = owner ]; then st=10; wu=3; fi
  timeout -k 10 500 python -u bench.py --workload $wl --steps $st --warmup $wu --no-cpu-baseline > gpurun_out/l2/bench_$wl.log 2>&1 || { tail -30 gpurun_out/l2/bench_$wl.log; exit 1; }
  echo "== $wl"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/l2/bench_$wl.log; grep -o '"kernel_ms_each": {[^}]*}' gpurun_out/l2/bench_$wl.log; grep -o '"parity_vs_oracle": [a-z]*' gpurun_out/l2/bench_$wl.log || true
done
