#!/bin/bash
# owner fold with LDS rule tables: suites + bench lines (r4k), phase clocks
# (r4l), one-stream node8 rocprof kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_r4k.sh && bash tools/gpu_r4l.sh || exit 1
export OSE_SKIP_BUILD=1
OUT=$R/gpurun_out/r4m; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
OSE_NODE8_ONE_STREAM=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/node8 -o ks -- python3 $R/bench.py --workload node8 --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $OUT/node8_prof.log 2>&1 || { echo "rocprof node8 failed"; tail -20 $OUT/node8_prof.log; exit 1; }
cd $R
f=$(ls $OUT/node8/*/ks_results.db $OUT/node8/ks_results.db 2>/dev/null | head -1); [ -n "$f" ] && python3 tools/rocpd_stats.py $f $OUT/node8_kernel_stats.csv > /dev/null
grep -o '"projected_ms_per_gpu_step": [0-9.]*' $OUT/node8_prof.log
head -16 $OUT/node8_kernel_stats.csv | cut -d, -f1-4
