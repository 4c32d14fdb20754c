# Round-4 closing tier: full GPU test tier, smoke, the headline bench, its windowed profile and
# the final-phase (3092-token) prefill profile.
set -o pipefail
TAG=${T:-r4final} STAGES="tests smoke bench profbench" STEPS=${STEPS:-5} TEST_TIMEOUT=1000 bash scripts/gpu/stages.sh || exit 1
TAG=${T:-r4final}pf3k STAGES=profpf TOKENS=3092 SEQS=1 bash scripts/gpu/stages.sh
