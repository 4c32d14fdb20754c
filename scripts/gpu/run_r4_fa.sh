set -o pipefail
TAG=r4fa1 STAGES="tests" PYTEST_ARGS="tests/test_kernels_gpu.py" PYTEST_K="prefill or flash or long" TEST_TIMEOUT=400 bash scripts/gpu/stages.sh || exit 1
TAG=r4fa1 STAGES=py PY_ARGS="scripts/gpu/microbench_prefill_attn.py" PY_TIMEOUT=300 bash scripts/gpu/stages.sh || exit 1
TAG=r4pf3k1 STAGES=profpf TOKENS=3092 SEQS=1 bash scripts/gpu/stages.sh || exit 1
