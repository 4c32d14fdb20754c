timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_wide_gemm.py tests/test_kernels_gpu.py -k "wide or skinny or qkv or gate_up or lm_head or splitk or preshuffled or fp8_decode" > gpurun_out/wide_tests.log 2>&1; tail -3 gpurun_out/wide_tests.log
timeout -k 10 120 python -u scripts/gpu/probe_skinny_mt.py --qkv-rope > gpurun_out/qkv_tail_on.txt 2>&1
ATTA_TAIL_SPLIT=0 timeout -k 10 120 python -u scripts/gpu/probe_skinny_mt.py --qkv-rope > gpurun_out/qkv_tail_off.txt 2>&1
echo "tail on"; tail -4 gpurun_out/qkv_tail_on.txt; echo "tail off"; tail -4 gpurun_out/qkv_tail_off.txt
timeout -k 10 400 python -u scripts/gpu/bench_wide.py --plans --m 33 64 85 128 > gpurun_out/wide_bench.txt 2>&1; cat gpurun_out/wide_bench.txt
timeout -k 10 300 python -u scripts/gpu/wide_timeline.py --m 85 > gpurun_out/wide_tl.txt 2>&1; cat gpurun_out/wide_tl.txt
