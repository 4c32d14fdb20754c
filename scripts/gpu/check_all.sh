#!/bin/bash
# Full GPU check: smoke(), kernel/engine tests, bf16 headline bench, fp8 bench (config-5 weights).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-6} $OUT/$name.log; if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=25 run pytest_gpu 1200 python -m pytest tests -m gpu -x -q -p no:cacheprovider
run bench_bf16 600 python bench.py --steps 2 --warmup 1 --verbose
run bench_fp8 600 python bench.py --steps 2 --warmup 1 --verbose --quantization fp8
