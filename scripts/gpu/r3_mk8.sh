#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -E "rows|ATT|QKV|step span" $OUT/$name.log; if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi; }
for c in 200 1000; do run r3_mk_prof_ctx$c 300 python scripts/gpu/mk_profile.py --steps 24 --rows 1 5 --ctx $c; done
