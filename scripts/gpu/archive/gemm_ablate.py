#!/usr/bin/env python3
"""Which side bounds a phase of the prefill GEMM main loop: the same plain bf16 GEMM
(M x N x K, data-parallel schedule) with the MFMAs, the LDS-DMA staging or the ds_reads
compiled out (ops.prefill_gemm_config(ablate=...), measurement-only kernel variants).
Prints us per call and us per 64-byte K phase per tile round.

    python scripts/gpu/gemm_ablate.py > profiles/r3_prefill_gemm_ablation.txt
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from agentic_traffic_testing_amd import ops  # noqa: E402


def main():
    dev = "cuda"
    shapes = [(2600, 28672, 4096), (2048, 8192, 4096), (4096, 4096, 4096)]
    print("# prefill GEMM ablation (bf16 plain, schedule dp / group_m 4); us per call; "
          "phase = 64 B of K per operand row (32 k); rounds = ceil(tiles / 256)")
    for M, N, K in shapes:
        ws = [(torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16) for _ in range(3)]
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        tiles = ((M + 255) // 256) * (N // 256)
        rounds = (tiles + 255) // 256
        line = f"M={M} N={N} K={K} tiles={tiles} rounds={rounds} |"
        for ab, name in [(0, "full"), (1, "no-mfma"), (4, "no-mfma-fulllines"), (2, "no-dma"),
                         (3, "no-dsread")]:
            ops.prefill_gemm_config("dp", 4, ab)
            for i in range(3):
                ops.prefill_gemm(x, ws[i % 3], out=out)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            it = 20
            for i in range(it):
                ops.prefill_gemm(x, ws[i % 3], out=out)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / it
            line += f" {name} {us:7.1f} us ({us / rounds / (K // 32):.3f} us/phase)"
        ops.prefill_gemm_config("hybrid", 4, 0)
        tf = 2.0 * M * N * K / 1e6
        print(line, flush=True)
    assert ops.prefill_gemm_error() == 0


if __name__ == "__main__":
    main()
