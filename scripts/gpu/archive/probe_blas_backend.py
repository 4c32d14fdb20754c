"""Prefill GEMM shapes (Llama-3.1-8B, M = 2600 tokens) under hipBLASLt vs rocBLAS
(torch.backends.cuda.preferred_blas_library), bf16, median of event-timed loops."""
import statistics
import torch


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / iters * 1000)
    return statistics.median(res)


M = 2600
shapes = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)]
for lib in ("cublaslt", "cublas"):
    torch.backends.cuda.preferred_blas_library(lib)
    row = f"{lib:9s}"
    tot = 0.0
    for name, n, k in shapes:
        x = torch.randn(M, k, dtype=torch.bfloat16, device="cuda")
        w = torch.randn(n, k, dtype=torch.bfloat16, device="cuda")
        r = torch.randn(M, n, dtype=torch.bfloat16, device="cuda")
        if name in ("o", "down"):
            t = timeit(lambda: r.addmm_(x, w.t()))
        else:
            t = timeit(lambda: torch.nn.functional.linear(x, w))
        tot += t
        row += f" | {name} {t:7.1f} us {2 * M * n * k / t / 1e6:6.0f} TF"
    print(row + f" | sum {tot:7.1f} us", flush=True)
