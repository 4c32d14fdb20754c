"""Prefill gate_up GEMM (Llama-3.1-8B: N 28672, K 4096) at synthesis-prompt M: one GEMM vs
N-split / M-split variants, hipBLASLt vs rocBLAS, with 4 rotating weight copies (940 MB, past
the Infinity Cache) so every call streams its weight cold.  us per full gate_up product."""
import statistics

import torch


def timeit(fn, iters=8):
    for _ in range(2):
        fn(0)
    torch.cuda.synchronize()
    res = []
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for i in range(iters):
            fn(i)
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / iters * 1000)
    return statistics.median(res)


N, K = 28672, 4096
ws = [torch.randn(N, K, dtype=torch.bfloat16, device="cuda") for _ in range(4)]
for lib in ("cublaslt", "cublas"):
    torch.backends.cuda.preferred_blas_library(lib)
    for M in (2600, 2816, 1300, 512):
        x = torch.randn(M, K, dtype=torch.bfloat16, device="cuda")
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        row = f"{lib:9s} M={M:5d}"
        t = timeit(lambda i: torch.mm(x, ws[i % 4].t(), out=out))
        row += f" | one {t:7.1f} us {2 * M * N * K / t / 1e6:5.0f} TF"
        for parts in (2, 4):
            n = N // parts
            t = timeit(lambda i: [torch.mm(x, ws[i % 4][j * n:(j + 1) * n].t(),
                                           out=out[:, j * n:(j + 1) * n])
                                  for j in range(parts)])
            row += f" | N/{parts} {t:7.1f} us"
        m2 = M // 2
        t = timeit(lambda i: [torch.mm(x[j * m2:(j + 1) * m2], ws[i % 4].t(),
                                       out=out[j * m2:(j + 1) * m2]) for j in range(2)])
        row += f" | M/2 {t:7.1f} us"
        print(row, flush=True)
