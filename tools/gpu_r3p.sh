#!/bin/bash
# URL parity with the separator-with-body stores and unaligned word reads,
# then their A/B (default: both; _noslash8: word reads only; _word2: neither)
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out/r3p
timeout -k 10 400 python -u -m pytest tests/test_url_random.py tests/test_url_kats.py tests/test_concurrency.py tests/test_unicode_regex.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3p/pytest.log 2>&1 || { tail -30 gpurun_out/r3p/pytest.log; exit 1; }
tail -1 gpurun_out/r3p/pytest.log
bash tools/gpu_ab.sh r3p_ab _noslash8,_word2 fused url || exit 1
