# instruction/stall counters of url_template_kernel under several ablation settings
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out/pmc3
cd /tmp && export TMPDIR=/tmp
N=${1:-2000000}
for ab in 0 3 121 1; do
  OSE_URL_ABLATE=$ab timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc3/a$ab -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --spans $N > $GRAFT_REPO_ROOT/gpurun_out/pmc3/a$ab.log 2>&1 || { echo "pmc ablate $ab failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc3/a$ab.log; exit 1; }
done
echo done
