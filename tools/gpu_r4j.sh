#!/bin/bash
# owner-side bucketed fold (ose_shard_decide): exchange/chunk GPU suites,
# the owner and node8 bench lines, one-stream node8 rocprof kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export OSE_SKIP_BUILD=1
OUT=$R/gpurun_out/r4j; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_exchange.py tests/test_sampling_chunks.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_x.log 2>&1 || { tail -60 $OUT/pytest_x.log; exit 1; }
tail -1 $OUT/pytest_x.log
timeout -k 10 400 python -u bench.py --workload owner --steps 10 --warmup 3 > $OUT/bench_owner.log 2>&1 || { tail -30 $OUT/bench_owner.log; exit 1; }
tail -1 $OUT/bench_owner.log
timeout -k 10 500 python -u bench.py --workload node8 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_node8.log 2>&1 || { tail -30 $OUT/bench_node8.log; exit 1; }
tail -1 $OUT/bench_node8.log
cd /tmp && export TMPDIR=/tmp
OSE_NODE8_ONE_STREAM=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/node8 -o ks -- python3 $R/bench.py --workload node8 --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $OUT/node8_prof.log 2>&1 || { echo "rocprof node8 failed"; tail -20 $OUT/node8_prof.log; exit 1; }
cd $R
f=$(ls $OUT/node8/*/ks_results.db $OUT/node8/ks_results.db 2>/dev/null | head -1); [ -n "$f" ] && python3 tools/rocpd_stats.py $f $OUT/node8_kernel_stats.csv > /dev/null
grep -o '"projected_ms_per_gpu_step": [0-9.]*' $OUT/node8_prof.log
head -12 $OUT/node8_kernel_stats.csv
