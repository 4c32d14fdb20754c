set -o pipefail
set -e
export PYTHONUNBUFFERED=1
export ATTA_GRAPH_META_COPY=1
PROF_NAME=r5prof_gaps_gcopy STEPS=1 WARMUP=1 bash scripts/gpu/profile_bench.sh > gpurun_out/r5prof_gaps_gcopy_run.txt 2>&1 || { tail -20 gpurun_out/r5prof_gaps_gcopy_run.txt; exit 1; }
sed -n '/wall span/,$p' gpurun_out/r5prof_gaps_gcopy_summary.txt
