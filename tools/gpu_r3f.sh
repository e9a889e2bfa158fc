#!/bin/bash
# dup-bucket A/B (C4 fused and C3 sampling), its GPU test, node8 kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3f
mkdir -p $OUT
cd $R
export OSE_SKIP_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_sampling_random.py -m gpu -x -q -k "dup_buckets or shuffled" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for b in 0 1; do
    for w in fused sampling; do
      OSE_DUP_BUCKETS=$b timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-parity > $OUT/bench_${w}_b${b}_$rep.log 2>&1 || { tail -20 $OUT/bench_${w}_b${b}_$rep.log; exit 1; }
      echo "$w b=$b rep=$rep $(grep -o '"ms_per_step": [0-9.]*\|"trace_eval_kernel": [0-9.]*\|"trace_dup_check": [0-9.]*' $OUT/bench_${w}_b${b}_$rep.log | tr '\n' ' ')"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
OSE_NODE8_ONE_STREAM=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof8 -o ks -- python3 $R/bench.py --workload node8 --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $OUT/prof8.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof8.log; exit 1; }
db=$(find $OUT/prof8 -name "*.db" | head -1)
if [ -n "$db" ]; then python3 $R/tools/rocpd_stats.py $db $OUT/node8_kernel_stats.csv > /dev/null && head -25 $OUT/node8_kernel_stats.csv; fi
