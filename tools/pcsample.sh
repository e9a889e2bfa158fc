#!/bin/bash
# Stochastic PC sampling of one bench workload's kernels (rocprofv3 beta),
# with the -gline-tables-only build (odigos_amd/build.py --variant _g
# -gline-tables-only) so samples carry source lines.
# usage: bash tools/pcsample.sh <tag> <workload> [spans]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; WL=$2; N=${3:-10000000}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export OSE_SKIP_BUILD=1 OSE_LIB_VARIANT=_g
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval 1048576 --output-format csv -d $OUT/ps_$WL -o ps -- \
  python3 $R/bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-parity --spans $N > $OUT/ps_$WL.log 2>&1
rc=$?
ls -la $OUT/ps_$WL/*/ 2>/dev/null | head
exit $rc
