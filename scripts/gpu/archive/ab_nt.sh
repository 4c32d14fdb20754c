#!/bin/bash
# A/B the decode weight-stream cache policy (nt vs default) on the real bench, then profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-4} $OUT/$name.log; if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi; }
run pytest_gpu 900 python -m pytest tests -m gpu -x -q
ATTA_NT_WEIGHTS=1 run bench_nt1 600 python bench.py --steps 2 --warmup 1 --verbose
ATTA_NT_WEIGHTS=0 run bench_nt0 600 python bench.py --steps 2 --warmup 1 --verbose
if [ "${PROFILE:-1}" = "1" ]; then echo "=== profile"; bash scripts/gpu/profile_bench.sh; fi
