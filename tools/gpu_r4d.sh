#!/bin/bash
# round-4 re-entry pass: GPU suite + smoke + C4/C2 lines with the lookup
# bitmaps, A/B against the round-start build (_r4base), the narrow-word
# A/B, issue/stall counters, PC sampling of the URL kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_check.sh r4d fused url || exit 1
bash tools/gpu_ab.sh r4d_lut _r4base fused url || exit 1
bash tools/gpu_ab.sh r4d_nn _nn sampling || exit 1
bash tools/pmc_r4.sh r4d_pmc || exit 1
bash tools/pcsample.sh r4d_ps url 10000000
