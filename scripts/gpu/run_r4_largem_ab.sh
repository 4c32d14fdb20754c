# Large-M routing A/B after the tuned library table: hand-written GEMM vs tuned hipBLASLt
# at the engine's padded row buckets (bf16), and the fp8 arm (library untuned).
set -o pipefail
TAG=r4lm_bf16 STAGES=gemm GEMM_ARGS="--m 2048 2560 3200 4096 --tuned auto --rounds 3" bash scripts/gpu/stages.sh || exit 1
TAG=r4lm_fp8 STAGES=gemm GEMM_ARGS="--m 512 1024 2048 3200 --fp8 --rounds 3" bash scripts/gpu/stages.sh || exit 1
