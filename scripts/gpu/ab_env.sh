#!/bin/bash
# A/B any environment knob on the fan-out bench (same box, one run each, in order).
# usage: bash scripts/gpu/ab_env.sh "ATTA_OPROJ_PREFETCH=0" "ATTA_OPROJ_PREFETCH=2" ...
#        ("" = defaults); BENCH_ARGS adds bench.py flags (e.g. "--quantization fp8").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  i=$((i + 1))
  env $cfg timeout -k 10 300 python bench.py --steps ${AB_STEPS:-2} --warmup 1 ${BENCH_ARGS:-} \
    > gpurun_out/abenv_$i.log 2>&1 || { echo "run $i ($cfg) failed"; exit 1; }
  v=$(grep -o '"value": [0-9.]*' gpurun_out/abenv_$i.log)
  t=$(grep -o '"p95_ttft_s": [0-9.]*' gpurun_out/abenv_$i.log)
  echo "[$cfg] $v $t"
done
