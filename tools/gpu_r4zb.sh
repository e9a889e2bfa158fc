#!/bin/bash
# round 5b: the one-pass rule-chunk kernel — its GPU tests, the sampling and
# size suites, then sampling_wide / sampling / fused bench lines
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r4zb}
mkdir -p $OUT
cd $R
export OSE_SKIP_BUILD=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_sampling_chunks.py tests/test_sampling_random.py tests/test_size.py tests/test_exchange.py tests/test_sampling_kats.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for wl in sampling_wide sampling fused zipf; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$wl.log 2>&1 || { tail -20 $OUT/bench_$wl.log; exit 1; }
  echo "$wl $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$wl.log) $(grep -o '"kernel_ms_each": {[^}]*}' $OUT/bench_$wl.log) $(grep -o '"parity[^}]*}' $OUT/bench_$wl.log | head -c 300)"
done
