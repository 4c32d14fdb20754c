#!/bin/bash
# A/B the per-projection decode wave table on the fan-out bench (same box, one run each).
# usage: bash scripts/gpu/ab_waves.sh "" "qkv.ps=8" "down.ps=16" ...   ("" = default table)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  i=$((i + 1))
  ATTA_DECODE_WAVES="$cfg" timeout -k 10 300 python bench.py --steps 2 --warmup 1 ${BENCH_ARGS:-} \
    > gpurun_out/ab_$i.log 2>&1 || { echo "run $i ($cfg) failed"; exit 1; }
  v=$(grep -o '"value": [0-9.]*' gpurun_out/ab_$i.log)
  echo "[$cfg] $v"
done
