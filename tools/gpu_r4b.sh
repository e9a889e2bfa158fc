#!/bin/bash
# correctness pass + bench lines + the FOLD_ENDS A/B (owner, zipf) + PC sampling
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_check.sh r4b fused node8 || exit 1
bash tools/gpu_ab.sh r4b_fe _fe owner zipf || exit 1
bash tools/pcsample.sh r4b_ps sampling 10000000 || exit 1
bash tools/pcsample.sh r4b_ps url 10000000
