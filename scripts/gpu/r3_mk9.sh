#!/bin/bash
# compact attention units in the persistent decode step: oracle tests, then the phase timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $OUT/$name.log; if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi; }
run probe_mall 240 python scripts/gpu/probe_mall.py
run mk_tests 400 python -m pytest -x -v --timeout 180 --timeout-method thread tests/test_engine.py -k megakernel
for c in 200 1000; do run r3_mk_prof_ctx$c 300 python scripts/gpu/mk_profile.py --steps 24 --rows 1 5 --ctx $c; grep -E "rows|ATT|QKV|step span" $OUT/r3_mk_prof_ctx$c.log; done
