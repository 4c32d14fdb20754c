set -o pipefail
set -e
ATTA_ATTN256_WAVES=16 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "decode" > gpurun_out/r5_attn16_tests.log 2>&1 || { tail -20 gpurun_out/r5_attn16_tests.log; exit 1; }
tail -1 gpurun_out/r5_attn16_tests.log
PT=256 CTXS="600;450,450,450,450,450;900,900,900,900,900;3500" ATTA_ATTN256_WAVES=16 timeout -k 10 300 python -u scripts/gpu/trace_decode_attention.py > gpurun_out/attn256_w16.txt 2>&1
PT=128 CTXS="600;450,450,450,450,450;900,900,900,900,900;3500" timeout -k 10 300 python -u scripts/gpu/trace_decode_attention.py > gpurun_out/attn128_w8b.txt 2>&1
paste -d'|' gpurun_out/attn128_w8b.txt gpurun_out/attn256_w16.txt | grep -v amdgpu | cut -c1-200
for i in 1 2; do for v in 128 256; do
ATTA_ATTN256_WAVES=16 timeout -k 10 600 python -u bench.py --steps 3 --warmup 2 --set decode_partition_tokens_small=$v > gpurun_out/r5_pt${v}_$i.log 2>&1
python -c "import json; d=json.loads(open('gpurun_out/r5_pt${v}_$i.log').read().strip().splitlines()[-1]); print('small partitions $v', d['value'], d['p50_ttft_s'])"
done; done
