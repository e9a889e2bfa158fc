#!/bin/bash
# a route past the LDS rule table (spilled route bytes): chunk, exchange and
# sampling suites, then the sampling / sampling_wide / fused lines
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export OSE_SKIP_BUILD=1
OUT=$R/gpurun_out/r4s; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_sampling_chunks.py tests/test_exchange.py tests/test_sampling_random.py tests/test_sampling_kats.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for w in sampling sampling_wide fused; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$w.log 2>&1 || { tail -30 $OUT/bench_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$w.log) $(grep -o '"kernel_ms_each": {[^}]*}' $OUT/bench_$w.log) $(grep -o '"parity_vs_oracle": [a-z]*' $OUT/bench_$w.log)"
done
