#!/bin/bash
# URL parity on the GPU with the unaligned-store assembly, then its A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out/r3o
timeout -k 10 400 python -u -m pytest tests/test_url_random.py tests/test_url_kats.py tests/test_concurrency.py tests/test_sampling_random.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3o/pytest.log 2>&1 || { tail -30 gpurun_out/r3o/pytest.log; exit 1; }
tail -1 gpurun_out/r3o/pytest.log
bash tools/gpu_ab.sh r3o_ab _nouaw fused url || exit 1
