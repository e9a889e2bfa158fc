#!/bin/bash
# A/B of two builds on one box: bench lines of the given workloads with the
# default library and with OSE_LIB_VARIANT=<variant> (odigos_amd/build.py
# --variant), alternating, each step time-limited.
# usage: bash tools/gpu_ab.sh <tag> <variant> <workload>...
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; VAR=$2; shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export OSE_SKIP_BUILD=1
for wl in "$@"; do
  for v in "" "$VAR" "" "$VAR"; do
    name=${wl}${v:-_default}
    OSE_LIB_VARIANT=$v timeout -k 10 400 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $OUT/bench_$name.log 2>&1 || { tail -20 $OUT/bench_$name.log; exit 1; }
    echo "$name $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$name.log) $(grep -o '"kernel_ms_each": {[^}]*}' $OUT/bench_$name.log | tr -d '\n' | cut -c1-400)"
  done
done
