set -o pipefail
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5prof_burst
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --steps 2 --warmup 5 > gpurun_out/r5prof_burst_bench.log 2>&1
for k in 0 1 2 3; do python3 scripts/gpu/step_breakdown.py $OUT --mt-min 3 --nth $k; done > gpurun_out/r5_burst_breakdown.txt 2>&1
cat gpurun_out/r5_burst_breakdown.txt
find $OUT -name "*kernel_trace.csv" -delete
