set -o pipefail
set -e
export PYTHONUNBUFFERED=1
for i in 1 2; do for v in 4 8; do
ATTA_FLASH_WAVES=$v timeout -k 10 600 python -u scripts/gpu/probe_fanout_ttft.py --episodes 4 --warmup 5 > gpurun_out/r5_fw${v}_$i.log 2>&1
echo "flash waves $v"; grep -E "burst|planning|final" gpurun_out/r5_fw${v}_$i.log | awk '{printf "%s %d %s; ", $3, $5-$7, $10}'; echo
done; done
