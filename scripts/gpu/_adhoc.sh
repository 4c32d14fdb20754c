set -o pipefail
set -e
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke_final3.log 2>&1
grep -v amdgpu gpurun_out/r5_smoke_final3.log | tail -1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r5_gpu_tier_final3.log 2>&1 || { tail -40 gpurun_out/r5_gpu_tier_final3.log; exit 1; }
tail -1 gpurun_out/r5_gpu_tier_final3.log
