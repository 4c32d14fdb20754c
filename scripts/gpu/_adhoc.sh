set -o pipefail
export PYTHONUNBUFFERED=1
run() {  # tag, env assignments...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 3 --warmup 2 > gpurun_out/sweep5b_$tag.log 2>&1 || return 1
  echo "$tag $* $(grep -o '"value": [0-9.]*' gpurun_out/sweep5b_$tag.log)"
}
run base_a ATTA_X=0 && run lm8_a ATTA_DECODE_WAVES=lm_head.ps=8 &&
run base_b ATTA_X=0 && run lm8_b ATTA_DECODE_WAVES=lm_head.ps=8 &&
run base_c ATTA_X=0 && run lm8_c ATTA_DECODE_WAVES=lm_head.ps=8
