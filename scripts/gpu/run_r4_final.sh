# Round-4 closing tier: full GPU test tier, smoke, the headline bench and its windowed profile.
set -o pipefail
TAG=r4final STAGES="tests smoke bench profbench" STEPS=${STEPS:-5} TEST_TIMEOUT=1000 bash scripts/gpu/stages.sh
