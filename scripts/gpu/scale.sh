#!/bin/bash
# First 8-GPU lease: the whole scaling curve in one call.  One JSON line per
# point on stdout and in gpurun_out/scale.jsonl; per-point logs (RCCL NCCL_DEBUG=INFO lines
# included) in gpurun_out/scale_logs/.  Points: DP 8B at N = 1 2 4 8, TP 8B at N = 2 4 8,
# 70B bf16 and fp8 at TP = 8, IPC one-/two-shot vs RCCL all-reduce over xGMI at W = 2 4 8.
# Every point has its own time limit; the first failure ends the sweep (scripts/gpu/scale.py).
#
#   bash scripts/gpu/scale.sh                 # GPU node
#   bash scripts/gpu/scale.sh --device cpu    # the CPU twin (gloo, tiny model)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
python3 -u scripts/gpu/scale.py --logdir gpurun_out/scale_logs "$@" | tee gpurun_out/scale.jsonl
