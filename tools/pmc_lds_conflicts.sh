#!/bin/bash
# LDS bank conflicts of url_plan_kernel (diagnostic instance) with and without
# the assembly's byte stores (OSE_URL_ABLATE 64) and the bitmap build (4)
R=$GRAFT_REPO_ROOT
export OSE_LIB_VARIANT=_diag   # build it first: python -m odigos_amd.build --variant _diag OSE_DIAG=1
mkdir -p $R/gpurun_out/ldsc
cd /tmp && export TMPDIR=/tmp
for ab in 4096 64 4; do
  OSE_URL_ABLATE=$ab timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/ldsc/a$ab -o pmc -- python3 $R/bench.py --workload url --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $R/gpurun_out/ldsc/a$ab.log 2>&1 || { echo "pass $ab failed"; tail -20 $R/gpurun_out/ldsc/a$ab.log; exit 1; }
  echo "== ablate $ab"; python3 $R/tools/pmc_summary.py $R/gpurun_out/ldsc/a$ab url_plan_kernel
done
