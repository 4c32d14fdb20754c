set -o pipefail
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_wide_gemm.py tests/test_kernels_gpu.py tests/test_engine.py > gpurun_out/r5_tests.log 2>&1; tail -3 gpurun_out/r5_tests.log
timeout -k 10 400 python -u scripts/gpu/bench_wide.py --m 33 64 85 128 > gpurun_out/wide_bench.txt 2>&1; cat gpurun_out/wide_bench.txt
timeout -k 10 300 python -u scripts/gpu/wide_timeline.py --m 85 > gpurun_out/wide_tl.txt 2>&1; cat gpurun_out/wide_tl.txt
timeout -k 10 600 python -u bench.py --steps 3 --warmup 5 > gpurun_out/r5_bench_a.log 2>&1; tail -1 gpurun_out/r5_bench_a.log
