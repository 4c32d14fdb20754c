#!/bin/bash
# rocprofv3 kernel trace + stats of one short bench run (no PMC counters here).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
NAME=${PROF_NAME:-prof}
OUT=gpurun_out/$NAME
rm -rf $OUT; mkdir -p $OUT
ATTA_WINDOW_MARKERS=1 timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --steps ${STEPS:-1} --warmup ${WARMUP:-0} ${BENCH_ARGS:-} > gpurun_out/${NAME}_bench.log 2>&1
rc=$?
echo "rc=$rc"; grep -E '^\{' gpurun_out/${NAME}_bench.log | tail -1
python3 scripts/gpu/summarize_trace.py $OUT --window stream_read_kernel > gpurun_out/${NAME}_summary.txt 2>&1
head -40 gpurun_out/${NAME}_summary.txt
find $OUT -name "*kernel_trace.csv" -delete
exit $rc
