"""Build the prefill library-GEMM solution table (PyTorch TunableOp format) for one model:
every projection's GEMM, exactly as the prefill forward calls it (qkv / gate_up F.linear,
o / down residual addmm_), at every row bucket of agentic_traffic_testing_amd.tuning up to
--max-rows, tuned with a rotating buffer past the Infinity Cache (cold weights, as a real
prefill streams them).  Writes agentic_traffic_testing_amd/tuning/tunableop_gfx950_<model>.csv
(or --out); the engine loads it lookup-only (EngineConfig.gemm_tuning).

    python scripts/gpu/tune_prefill_gemms.py --model llama-3.1-8b --max-rows 8192
    python scripts/gpu/tune_prefill_gemms.py --model llama-3-70b --tp 8 --buckets 16,96,384
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from agentic_traffic_testing_amd import tuning  # noqa: E402
from agentic_traffic_testing_amd.config import resolve_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3.1-8b")
    ap.add_argument("--max-rows", type=int, default=8192)
    ap.add_argument("--min-rows", type=int, default=1)
    ap.add_argument("--out", default="")
    ap.add_argument("--duration-ms", type=int, default=40,
                    help="TunableOp time per candidate solution")
    ap.add_argument("--tp", type=int, default=1,
                    help="tune the per-rank shard shapes of this TP degree (column-parallel "
                         "qkv / gate_up: N / tp; row-parallel o / down: K / tp)")
    ap.add_argument("--fp8", action="store_true",
                    help="tune the fp8 prefill GEMMs (row-wise scaled torch._scaled_mm, as "
                         "ops.gemm_fp8 calls it) instead of the bf16 ones")
    ap.add_argument("--buckets", default="",
                    help="comma-separated row buckets instead of every bucket in range")
    a = ap.parse_args()
    mc = resolve_model(a.model)[0]
    out = a.out or str(tuning.table_path(mc.name))
    tp = a.tp
    H, I = mc.hidden_size, mc.intermediate_size
    qkv_n = (mc.num_heads + 2 * mc.num_kv_heads) * mc.head_dim
    o_k = mc.num_heads * mc.head_dim
    assert qkv_n % tp == 0 and o_k % tp == 0 and I % tp == 0, "shapes not divisible by --tp"
    shapes = {"qkv": (qkv_n // tp, H, False), "o": (H, o_k // tp, True),
              "gate_up": (2 * I // tp, H, False), "down": (H, I // tp, True)}
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.record_untuned_enable(False)
    tun.set_filename(out)
    tun.set_max_tuning_duration(a.duration_ms)
    tun.set_rotating_buffer_size(512)  # MB: candidates run on rotating operand copies
    buckets = ([int(b) for b in a.buckets.split(",")] if a.buckets else
               [b for b in tuning.all_buckets(a.max_rows) if b >= a.min_rows])
    assert all(tuning.bucket_rows(b) == b for b in buckets), "not a row bucket"
    print(f"# tuning {a.model} TP={tp}: {len(shapes)} projections x {len(buckets)} row buckets "
          f"({buckets[0]}..{buckets[-1]}) -> {out}", flush=True)
    t0 = time.time()
    ws = {k: (torch.rand(n, kk, device="cuda") * 2 - 1).to(torch.bfloat16) / kk ** 0.5
          for k, (n, kk, _) in shapes.items()}
    f8 = torch.float8_e4m3fn
    w8 = {k: (w.float() * 8).to(f8) for k, w in ws.items()} if a.fp8 else {}
    for m in buckets:
        for name, (n, k, res) in shapes.items():
            x = (torch.rand(m, k, device="cuda") * 2 - 1).to(torch.bfloat16)
            if a.fp8:
                torch._scaled_mm(x.to(f8), w8[name].t(),
                                 scale_a=torch.rand(m, 1, device="cuda") + 0.5,
                                 scale_b=torch.rand(1, n, device="cuda") + 0.5,
                                 out_dtype=torch.bfloat16)
            elif res:
                r = torch.zeros(m, n, device="cuda", dtype=torch.bfloat16)
                r.addmm_(x, ws[name].t())
            else:
                torch.nn.functional.linear(x, ws[name])
        torch.cuda.synchronize()
        print(f"  M={m:5d} tuned ({time.time() - t0:6.1f} s)", flush=True)
    # the results file is written when TunableOp's context is torn down (process exit);
    # report what was found now
    n = sum(1 for v in tun.get_results()) if hasattr(tun, "get_results") else -1
    print(f"# {n} tuned entries", flush=True)


if __name__ == "__main__":
    main()
