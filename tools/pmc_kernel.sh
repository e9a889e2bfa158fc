# Issue/stall PMC counters of one bench workload's kernels (separate --pmc
# passes, kernel-trace only; MI355X_MICROARCH.md rocprofv3 PMC slots).
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
WL=${1:-sampling}
N=${2:-10000000}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$WL
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $OUT/p$i -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --spans $N > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
done
for k in ${3:-trace_eval_kernel}; do echo "== $k"; python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT $k; done
