#!/bin/bash
# plan fallbacks moved to url_plan_slow_kernel: URL GPU tests (KATs incl. long segments), clocks, C2/C4/C5 benches
set -o pipefail
mkdir -p gpurun_out/sp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_url_kats.py tests/test_url_random.py tests/test_size.py tests/test_concurrency.py > gpurun_out/sp/tests.log 2>&1
rc=$?
tail -3 gpurun_out/sp/tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/sp/tests.log | head -30; exit $rc; fi
for wl in url fused zipf; do
  timeout -k 10 500 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/sp/bench_$wl.log 2>&1 || { tail -30 gpurun_out/sp/bench_$wl.log; exit 1; }
  echo "== $wl"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/sp/bench_$wl.log; grep -o '"kernel_ms_each": {[^}]*}' gpurun_out/sp/bench_$wl.log; grep -o '"parity_vs_oracle": [a-z]*' gpurun_out/sp/bench_$wl.log
done
