#!/bin/bash
# round-4 closing pass B: PMC HBM traffic per workload (separate FETCH/WRITE
# passes) and the rocprof kernel stats of the C4 line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for wl in fused url sampling zipf; do bash tools/pmc_traffic.sh $wl || exit 1; done
export OSE_SKIP_BUILD=1
OUT=$R/gpurun_out/r4z; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/fused -o ks -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $OUT/fused_prof.log 2>&1 || { echo "rocprof fused failed"; tail -20 $OUT/fused_prof.log; exit 1; }
cd $R
f=$(ls $OUT/fused/*/ks_results.db $OUT/fused/ks_results.db 2>/dev/null | head -1); [ -n "$f" ] && python3 tools/rocpd_stats.py $f $OUT/fused_kernel_stats.csv > /dev/null
head -8 $OUT/fused_kernel_stats.csv | cut -d, -f1-4
cat gpurun_out/pmc_traffic_*.json | head -c 3000
