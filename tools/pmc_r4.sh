#!/bin/bash
# Issue / stall / LDS counters of the C4 kernels and of C2's url_plan at 10M
# spans (separate --pmc passes, kernel-trace only).
# usage: bash tools/pmc_r4.sh <tag> [lib variant]
set -o pipefail
export OSE_SKIP_BUILD=1
export OSE_LIB_VARIANT=${2:-}
R=$GRAFT_REPO_ROOT
TAG=${1:-pmc_r4}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
P3="SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA"
run() { # wl pass counters
  timeout -s KILL 150 rocprofv3 --pmc $3 --kernel-trace --output-format csv -d $OUT/$1_$2 -o pmc -- python3 $R/bench.py --workload $1 --steps 2 --warmup 1 --no-cpu-baseline --no-parity --spans 10000000 > $OUT/$1_$2.log 2>&1 || { echo "pmc pass $1 $2 failed"; tail -20 $OUT/$1_$2.log; return 1; }
}
run fused p1 "$P1" && run fused p2 "$P2" && run url p1 "$P1" && run url p2 "$P2" || exit 1
run fused p3 "$P3" && run url p3 "$P3"
for k in url_plan_kernel trace_eval_kernel url_copy_kernel; do echo "== fused $k"; python3 $R/tools/pmc_summary.py "$OUT/fused_*" $k; done
echo "== url url_plan_kernel"; python3 $R/tools/pmc_summary.py "$OUT/url_*" url_plan_kernel
