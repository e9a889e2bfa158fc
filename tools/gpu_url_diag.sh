# URL kernel diagnostics: per-section shader clocks and issue/stall PMC counters (C2, 10M spans)
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/url_clocks.py 10000000 8 > gpurun_out/url_clocks.log 2>&1 || { echo "clocks failed"; tail -20 gpurun_out/url_clocks.log; exit 1; }
cat gpurun_out/url_clocks.log | grep -v amdgpu.ids
timeout -k 10 600 bash tools/pmc_kernel.sh url 10000000 "url_plan_kernel url_emit_kernel" > gpurun_out/url_pmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/url_pmc.log; exit 1; }
cat gpurun_out/url_pmc.log
