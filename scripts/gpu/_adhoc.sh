set -o pipefail
set -e
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/gpu/probe_graph_gap.py > gpurun_out/r5_graph_gap.txt 2>&1
grep -v amdgpu gpurun_out/r5_graph_gap.txt
