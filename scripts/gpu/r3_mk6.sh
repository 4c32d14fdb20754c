#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-8} $OUT/$name.log; if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi; }
ATTA_MK_LOADERS=0 TAILN=4 run r3_mk_tests_rs 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_engine.py -k "megakernel"
ATTA_MK_LOADERS=0 TAILN=22 run r3_mk_prof_rs 300 python scripts/gpu/mk_profile.py --steps 24 --rows 1 5
TAILN=4 run r3_mk_tests_ring 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_engine.py -k "megakernel"
