# Host- vs GPU-bound check of the cached-prompt prefills (17 rows planning, 85 rows burst):
# wall time per prefill (prefill_bench) against windowed kernel time (rocprofv3).
set -o pipefail
TAG=r4sp17 STAGES=profpf TOKENS=17 SEQS=1 REPS=10 bash scripts/gpu/stages.sh || exit 1
TAG=r4sp85 STAGES=profpf TOKENS=85 SEQS=5 REPS=10 bash scripts/gpu/stages.sh || exit 1
