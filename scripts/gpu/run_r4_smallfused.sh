# <= 32-row prefill steps on the fused decode kernels: full GPU test tier, the 17-row prefill
# profile, and the cached-prompt bench (20-step driver regime shortened: 6 steps after 5
# warm-ups) with the path on and off.
set -o pipefail
TAG=r4sf STAGES=tests TEST_TIMEOUT=900 bash scripts/gpu/stages.sh || exit 1
TAG=r4sf17 STAGES=profpf TOKENS=17 SEQS=1 REPS=10 bash scripts/gpu/stages.sh || exit 1
TAG=r4sf_on STAGES=bench STEPS=6 BENCH_ARGS="--warmup 5" bash scripts/gpu/stages.sh || exit 1
TAG=r4sf_off STAGES=bench STEPS=6 BENCH_ARGS="--warmup 5 --set small_prefill_fused=0" bash scripts/gpu/stages.sh || exit 1
