#!/bin/bash
# round-4 pass: GPU suite + smoke + C4/C2 lines with the lookup bitmaps, A/B
# against the round-start build (_r4base), rocprof kernel stats of C4 and of
# the one-stream node8 step, issue/stall counters, PC sampling of url_plan
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export OSE_SKIP_BUILD=1
bash tools/gpu_check.sh r4e fused url sampling zipf owner || exit 1
bash tools/gpu_ab.sh r4e_nn _nn sampling fused || exit 1
OUT=$R/gpurun_out/r4e_prof; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/fused -o ks -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $OUT/fused.log 2>&1 || { echo "rocprof fused failed"; tail -20 $OUT/fused.log; exit 1; }
OSE_NODE8_ONE_STREAM=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/node8 -o ks -- python3 $R/bench.py --workload node8 --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $OUT/node8.log 2>&1 || { echo "rocprof node8 failed"; tail -20 $OUT/node8.log; exit 1; }
cd $R
for d in fused node8; do f=$(ls $OUT/$d/*/ks_results.db $OUT/$d/ks_results.db 2>/dev/null | head -1); [ -n "$f" ] && python3 tools/rocpd_stats.py $f $OUT/${d}_kernel_stats.csv > /dev/null; done
bash tools/pmc_r4.sh r4e_pmc || exit 1
bash tools/pcsample.sh r4e_ps url 10000000
bash tools/pcsample.sh r4e_ps sampling 10000000
