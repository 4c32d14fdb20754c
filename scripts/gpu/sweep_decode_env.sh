# Bench-level A/B of decode GEMV knobs through their env overrides (same box, back to back):
# split-K and waves per projection (ops.DECODE_KSPLIT / ops.DECODE_WAVES).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
run() {  # tag, env assignments...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 2 --warmup 1 > gpurun_out/sweep_$tag.log 2>&1 || return 1
  echo "$tag $* $(grep -o '"value": [0-9.]*' gpurun_out/sweep_$tag.log)"
}
run base ATTA_X=0 &&
run qkv_ks2 ATTA_DECODE_KSPLIT=qkv=2 &&
run o_ks2 ATTA_DECODE_KSPLIT=o=2 &&
run qkv_w8 ATTA_DECODE_WAVES=qkv.ps=8 &&
run o_w16 ATTA_DECODE_WAVES=o.ps=16 &&
run base2 ATTA_X=0
