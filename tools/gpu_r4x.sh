#!/bin/bash
# one-stream node8 rocprof kernel stats (pack scatter after the route-tail branch)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export OSE_SKIP_BUILD=1
OUT=$R/gpurun_out/r4x; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
OSE_NODE8_ONE_STREAM=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/node8 -o ks -- python3 $R/bench.py --workload node8 --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $OUT/node8.log 2>&1 || { echo "rocprof node8 failed"; tail -20 $OUT/node8.log; exit 1; }
cd $R
f=$(ls $OUT/node8/*/ks_results.db $OUT/node8/ks_results.db 2>/dev/null | head -1); [ -n "$f" ] && python3 tools/rocpd_stats.py $f $OUT/node8_kernel_stats.csv > /dev/null
grep -o '"projected_ms_per_gpu_step": [0-9.]*' $OUT/node8.log
grep -E "shard_scatter|shard_hist|owner_|url_plan" $OUT/node8_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 300 python -u bench.py --workload sampling --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $OUT/sampling.log 2>&1 && grep -o '"kernel_ms_each": {[^}]*}' $OUT/sampling.log
