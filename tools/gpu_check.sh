# GPU iteration: gpu tests, ablation timings, bench (each step time-limited)
set -o pipefail
cd $GRAFT_REPO_ROOT
export OSE_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/ablate_url.py > gpurun_out/ablate.log 2>&1 || { echo "ablate failed"; tail -20 gpurun_out/ablate.log; exit 1; }
cat gpurun_out/ablate.log | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
grep '"metric"' gpurun_out/bench.log
