#!/bin/bash
# round-4 profiles: rocprof kernel stats of C4 and of the one-stream node8
# step, the drop-in (PCIe-inclusive) timings
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export OSE_SKIP_BUILD=1
OUT=$R/gpurun_out/r4p; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/fused -o ks -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $OUT/fused.log 2>&1 || { echo "rocprof fused failed"; tail -20 $OUT/fused.log; exit 1; }
OSE_NODE8_ONE_STREAM=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/node8 -o ks -- python3 $R/bench.py --workload node8 --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $OUT/node8.log 2>&1 || { echo "rocprof node8 failed"; tail -20 $OUT/node8.log; exit 1; }
cd $R
for d in fused node8; do f=$(ls $OUT/$d/*/ks_results.db $OUT/$d/ks_results.db 2>/dev/null | head -1); [ -n "$f" ] && python3 tools/rocpd_stats.py $f $OUT/${d}_kernel_stats.csv > /dev/null; done
grep -o '"projected_ms_per_gpu_step": [0-9.]*' $OUT/node8.log
head -8 $OUT/fused_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 400 python -u tools/dropin_bench.py --out $OUT/dropin.json > $OUT/dropin.log 2>&1 || { tail -20 $OUT/dropin.log; exit 1; }
tail -c 1500 $OUT/dropin.json
