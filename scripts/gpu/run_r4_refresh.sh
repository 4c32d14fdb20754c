# Refresh the secondary configurations on the final round-4 tree.
set -o pipefail
TAG=r4fin STAGES=http STEPS=3 bash scripts/gpu/stages.sh || exit 1
TAG=r4fin_fp8 STAGES=bench STEPS=2 BENCH_ARGS="--quantization fp8" bash scripts/gpu/stages.sh || exit 1
TAG=r4fin_70bfp8 STAGES=bench STEPS=1 BENCH_ARGS="--model llama-3-70b --quantization fp8" bash scripts/gpu/stages.sh || exit 1
