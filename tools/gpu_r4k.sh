#!/bin/bash
# chunked rule lists through partial records (sample_by_records): chunk and
# exchange GPU suites, sampling_wide / owner / node8 bench lines
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export OSE_SKIP_BUILD=1
OUT=$R/gpurun_out/r4k; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_sampling_chunks.py tests/test_exchange.py tests/test_span_attribute.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_x.log 2>&1 || { tail -60 $OUT/pytest_x.log; exit 1; }
tail -1 $OUT/pytest_x.log
for w in sampling_wide owner; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 10 --warmup 3 > $OUT/bench_$w.log 2>&1 || { tail -30 $OUT/bench_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$w.log) $(grep -o '"kernel_ms_each": {[^}]*}' $OUT/bench_$w.log) $(grep -o '"parity_vs_oracle": [a-z]*' $OUT/bench_$w.log)"
done
timeout -k 10 500 python -u bench.py --workload node8 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_node8.log 2>&1 || { tail -30 $OUT/bench_node8.log; exit 1; }
grep -o '"projected_ms_per_gpu_step": [0-9.]*\|"parity_vs_oracle": [a-z]*' $OUT/bench_node8.log
