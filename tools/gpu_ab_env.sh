#!/bin/bash
# A/B of environment settings on one box: bench lines of one workload with
# each "NAME=VALUE[:NAME=VALUE...]" setting ("-" = none), interleaved twice,
# each step time-limited.
# usage: bash tools/gpu_ab_env.sh <tag> <workload> <setting>...
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; WL=$2; shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export OSE_SKIP_BUILD=1
for rep in 1 2; do
  for st in "$@"; do
    name=${WL}_$(echo "$st" | tr -c 'A-Za-z0-9_\n' '_')_$rep
    envs=()
    [ "$st" != "-" ] && IFS=':' read -ra envs <<< "$st"
    env "${envs[@]}" timeout -k 10 400 python -u bench.py --workload $WL --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $OUT/bench_$name.log 2>&1 || { tail -20 $OUT/bench_$name.log; exit 1; }
    echo "$name $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$name.log) $(grep -o '"kernel_ms_each": {[^}]*}' $OUT/bench_$name.log | grep -o '"[a-z_]*": [0-9.]*[1-9][0-9.]*' | tr '\n' ' ')"
  done
done
