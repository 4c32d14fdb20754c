"""Probe: prefill GEMMs of Llama-3.1-8B at several M, hipBLASLt default vs TunableOp-selected
(rocBLAS + hipBLASLt solutions benchmarked per shape).  Prints us per GEMM set (qkv, o+res,
gate_up, down+res) for each M."""
import os
import statistics
import sys
import time

import torch

M_LIST = [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else "128,256,384,512,1024,2600,2816").split(",")]
H, I, QKV = 4096, 14336, 6144


def run(M, iters=20):
    x = torch.randn(M, H, device="cuda", dtype=torch.bfloat16)
    a = torch.randn(M, 4096, device="cuda", dtype=torch.bfloat16)
    g = torch.randn(M, I, device="cuda", dtype=torch.bfloat16)
    r = torch.randn(M, H, device="cuda", dtype=torch.bfloat16)
    wq = torch.randn(QKV, H, device="cuda", dtype=torch.bfloat16)
    wo = torch.randn(H, 4096, device="cuda", dtype=torch.bfloat16)
    wg = torch.randn(2 * I, H, device="cuda", dtype=torch.bfloat16)
    wd = torch.randn(H, I, device="cuda", dtype=torch.bfloat16)

    def step():
        torch.nn.functional.linear(x, wq)
        r.addmm_(a, wo.t())
        torch.nn.functional.linear(x, wg)
        r.addmm_(g, wd.t())
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        for _ in range(iters):
            step()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) / iters * 1e6)
    flops = 2 * M * H * (QKV + 4096 + 2 * I + I)
    t = statistics.median(ts)
    return t, flops / t / 1e6


if __name__ == "__main__":
    tag = os.environ.get("TAG", "default")
    for M in M_LIST:
        t, tf = run(M)
        print(f"{tag:8s} M={M:5d}: {t:8.1f} us per layer of GEMMs  {tf:6.0f} TFLOP/s", flush=True)
