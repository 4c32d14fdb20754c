#!/bin/bash
# batched partition-merge loads in the persistent decode step: oracle tests, phase timeline,
# end-to-end bench with the megakernel on
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $OUT/$name.log; if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi; }
run mk_tests 400 python -m pytest -x -q --timeout 180 --timeout-method thread tests/test_engine.py -k megakernel
for c in 1000 3000; do run r3_mk_prof_ctx$c 300 python scripts/gpu/mk_profile.py --steps 24 --rows 1 5 --ctx $c; grep -E "rows|ATT|QKV|step span|err" $OUT/r3_mk_prof_ctx$c.log; done
run bench_mk 400 python bench.py --steps 2 --warmup 1 --set decode_megakernel=1
grep -E '^\{' $OUT/bench_mk.log | cut -c1-200
