#!/bin/bash
# A/B of builds on one box: bench lines of the given workloads with the
# default library and with each OSE_LIB_VARIANT (odigos_amd/build.py
# --variant), interleaved twice, each step time-limited.
# usage: bash tools/gpu_ab.sh <tag> <variant[,variant...]> <workload>...
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; VARS=$2; shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export OSE_SKIP_BUILD=1
for wl in "$@"; do
  for rep in 1 2; do
    for v in "" ${VARS//,/ }; do
      name=${wl}${v:-_default}_$rep
      OSE_LIB_VARIANT=$v timeout -k 10 400 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $OUT/bench_$name.log 2>&1 || { tail -20 $OUT/bench_$name.log; exit 1; }
      echo "$name $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$name.log) $(grep -o '"kernel_ms_each": {[^}]*}' $OUT/bench_$name.log | grep -o '"url_plan_kernel": [0-9.]*\|"trace_multi_kernel": [0-9.]*\|"trace_eval_kernel": [0-9.]*\|"trace_dup_check": [0-9.]*\|"trace_long_kernel": [0-9.]*\|"trace_run_list": [0-9.]*\|"url_copy_kernel": [0-9.]*\|"size_[a-z]*_kernel": [0-9.]*' | tr '\n' ' ')"
    done
  done
done
