#!/bin/bash
# url_copy prefetch A/B (C4, C5)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab.sh r3n_ab _cpf,_nocpf fused zipf || exit 1
