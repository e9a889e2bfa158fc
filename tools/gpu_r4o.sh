#!/bin/bash
# round-4 pass on the committed build: GPU suite, smoke, every bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_check.sh r4o fused url sampling zipf owner node8 sampling_wide
