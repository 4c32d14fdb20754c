set -o pipefail
TAG=r4ew STAGES=py PY_ARGS="scripts/gpu/probe_elementwise.py --m 382 3200" PY_TIMEOUT=200 bash scripts/gpu/stages.sh || exit 1
TAG=r4fa STAGES=py PY_ARGS="scripts/gpu/microbench_prefill_attn.py" PY_TIMEOUT=300 bash scripts/gpu/stages.sh || exit 1
TAG=r4route STAGES=bench STEPS=2 bash scripts/gpu/stages.sh || exit 1
