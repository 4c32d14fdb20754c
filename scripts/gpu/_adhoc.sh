set -o pipefail
set -e
export PYTHONUNBUFFERED=1
for i in 1 2; do for v in 1 3 5; do
ATTA_WIDE_PLAN_RED_US=$v timeout -k 10 600 python -u scripts/gpu/probe_fanout_ttft.py --episodes 4 --warmup 5 > gpurun_out/r5_red${v}_$i.log 2>&1
echo "reduce cost $v us"; grep -E "burst|planning" gpurun_out/r5_red${v}_$i.log | awk '{printf "%s %d %s; ", $3, $5-$7, $10}'; echo
done; done
