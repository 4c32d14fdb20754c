set -o pipefail
set -e
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5_driverlike_final3.log 2>&1
tail -1 gpurun_out/r5_driverlike_final3.log
