# stall breakdown for url_template_kernel (separate --pmc passes, kernel-trace only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp
N=${1:-2000000}
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
            "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_IFETCH_LEVEL GRBM_GUI_ACTIVE" \
            "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT" \
            "SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LEVEL_WAVES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc2/p$i -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --spans $N > $GRAFT_REPO_ROOT/gpurun_out/pmc2/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc2/p$i.log; exit 1; }
done
echo done
