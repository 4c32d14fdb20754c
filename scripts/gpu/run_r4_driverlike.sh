# The driver's headline invocation (bench.py --gpus 1 --steps 20 --warmup 5) on the final tree.
set -o pipefail
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_driverlike_bench.log 2>&1; rc=$?; tail -2 gpurun_out/r4_driverlike_bench.log; exit $rc
