#!/bin/bash
# GPU-box check: kernel/engine tests, smoke, short bench.  Every GPU step has its own
# time limit; a crash / fault / timeout (anything but a plain test failure) stops the run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-2}
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a $OUT/summary.txt
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $OUT/summary.txt
  tail -4 $OUT/$name.log | tee -a $OUT/summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)" | tee -a $OUT/summary.txt; exit $rc; fi
  return 0
}
step pytest_gpu 1200 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 900 python bench.py --steps $STEPS --warmup 1 --verbose
