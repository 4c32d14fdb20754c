set -o pipefail
TAG=${T:-r4fa3} STAGES="tests" PYTEST_ARGS="tests/test_kernels_gpu.py" PYTEST_K="prefill or flash or long or norm" TEST_TIMEOUT=400 bash scripts/gpu/stages.sh || exit 1
TAG=${T:-r4fa3} STAGES=py PY_ARGS="scripts/gpu/microbench_prefill_attn.py --impls flash" PY_TIMEOUT=300 bash scripts/gpu/stages.sh || exit 1
TAG=${T:-r4fa3}ew STAGES=py PY_ARGS="scripts/gpu/probe_elementwise.py --m 73 382 3200" PY_TIMEOUT=200 bash scripts/gpu/stages.sh || exit 1
FA_TAG=${FA_TAG:-3} bash scripts/gpu/run_r4_fa_pmc.sh
