#!/bin/bash
# Round-3 pass: suite, smoke, default bench line, rocprof stats (gpu_round3.sh),
# then the quarter-row A/B on C4 and C2.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round3.sh r3l || exit 1
bash tools/gpu_ab.sh r3l_ab _qrows fused url || exit 1
