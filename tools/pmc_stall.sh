#!/bin/bash
# stall / issue breakdown of the C4 kernels (separate --pmc passes, kernel-trace only)
set -o pipefail
export OSE_SKIP_BUILD=1
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc3
cd /tmp && export TMPDIR=/tmp
N=${1:-10000000}
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $R/gpurun_out/pmc3/p$i -o pmc -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --spans $N > $R/gpurun_out/pmc3/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $R/gpurun_out/pmc3/p$i.log; exit 1; }
done
for k in url_plan_kernel trace_eval_kernel url_copy_kernel size_tail_kernel; do echo "== $k"; python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc3 $k; done
