#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TESTS="tests/test_sampling_random.py tests/test_sampling_kats.py tests/test_sampling_chunks.py" bash tools/gpu_check.sh r4c || exit 1
bash tools/gpu_ab.sh r4c_nn _nn sampling fused || exit 1
bash tools/gpu_ab.sh r4c_fe _fe owner zipf || exit 1
bash tools/pcsample.sh r4c_ps sampling 10000000 || exit 1
bash tools/pcsample.sh r4c_ps url 10000000
