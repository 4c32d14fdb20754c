#!/bin/bash
# rocprofv3 kernel trace + stats of one short bench run (no PMC counters here).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --steps ${STEPS:-1} --warmup ${WARMUP:-0} ${BENCH_ARGS:-} > gpurun_out/prof_bench.log 2>&1
rc=$?
echo "rc=$rc"; grep -E '^\{' gpurun_out/prof_bench.log | tail -1
python3 scripts/gpu/summarize_trace.py $OUT > gpurun_out/prof_summary.txt 2>&1
head -40 gpurun_out/prof_summary.txt
find $OUT -name "*kernel_trace.csv" -delete
exit $rc
