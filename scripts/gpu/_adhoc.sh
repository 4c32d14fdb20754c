set -o pipefail
set -e
export PYTHONUNBUFFERED=1
for i in 1 2; do for v in "0,0" "49,120" "33,120"; do
ATTA_O_LIBRARY_ROWS=$v timeout -k 10 600 python -u scripts/gpu/probe_fanout_ttft.py --episodes 4 --warmup 5 > gpurun_out/r5_olib_${v/,/_}_$i.log 2>&1
echo "o-library rows $v"; grep -E "burst|planning" gpurun_out/r5_olib_${v/,/_}_$i.log | awk '{printf "%s %d %s; ", $3, $5-$7, $10}'; echo
done; done
