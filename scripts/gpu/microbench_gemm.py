"""Decode GEMM microbenchmark: MFMA skinny GEMM vs hipBLASLt (F.linear) at the Llama-3-8B
decode shapes; reports us and effective HBM GB/s (weights streamed once)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from agentic_traffic_testing_amd import ops  # noqa: E402

SHAPES = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096),
          ("down", 4096, 14336), ("lm_head", 128256, 4096)]


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    # rotate weights so they are not L2/MALL resident
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000


def main():
    assert ops.native_available()
    print(f"{'shape':>8} {'M':>3} {'blaslt_us':>10} {'GB/s':>7} {'skinny4_us':>11} {'GB/s':>7} {'skinny8_us':>11} {'GB/s':>7}")
    for name, n, k in SHAPES:
        ws = [torch.randn(n, k, dtype=torch.bfloat16, device="cuda") * 0.02 for _ in range(4)]
        nbytes = n * k * 2
        for m in (1, 5, 12, 16):
            x = torch.randn(m, k, dtype=torch.bfloat16, device="cuda")
            out = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
            i = [0]

            def blas():
                i[0] = (i[0] + 1) % 4
                torch.nn.functional.linear(x, ws[i[0]])

            def sk(waves):
                def f():
                    i[0] = (i[0] + 1) % 4
                    torch.ops.atta.skinny_gemm(out, x, ws[i[0]], None, waves)
                return f
            tb = timeit(blas)
            t4 = timeit(sk(4))
            t8 = timeit(sk(8))
            print(f"{name:>8} {m:3d} {tb:10.1f} {nbytes / tb / 1e3:7.0f} {t4:11.1f} {nbytes / t4 / 1e3:7.0f} {t8:11.1f} {nbytes / t8 / 1e3:7.0f}", flush=True)


if __name__ == "__main__":
    main()
