"""Wide small-M GEMM (ops/csrc/wide.hip) vs the library at the Llama-3.1-8B projection shapes:
us per call and weight-stream TB/s, cold weights (rotating copies past the 256 MB Infinity
Cache), with the fused epilogues the engine uses (qkv: norm + RoPE + K/V write, o / down:
residual add, gate_up: norm + SiLU-mul).  Library column = F.linear (hipBLASLt) on row-major
weights plus the separate norm / RoPE / SiLU kernels it needs.

    python scripts/gpu/bench_wide.py [--m 33 85 128] [--plans] [--graph]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from agentic_traffic_testing_amd import ops  # noqa: E402
from agentic_traffic_testing_amd.ops import reference as ref  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
# Llama-3-70B TP=1 (--model 70b): 64 q / 8 kv heads, hidden 8192, FFN 28672
SHAPES_70B = {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192),
              "down": (8192, 28672)}
PLANS = {"qkv": [(6, 4), (8, 4), (6, 2), (4, 4), (8, 6)],
         "o": [(8, 8), (4, 4), (8, 4), (4, 8), (6, 6)],
         "gate_up": [(7, 1), (8, 1), (4, 1), (4, 2), (8, 2)],
         "down": [(8, 8), (4, 4), (8, 4), (4, 8), (8, 16)]}


GRAPH = False


def timeit(fn, n=30, reps=3):
    """us per call over n back-to-back calls; with --graph the n calls are captured in one
    hipGraph and replayed (GPU time incl. launch gaps, no host launch cost - the decode
    step's regime), else launched eagerly (the prefill step's regime)."""
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    g = None
    if GRAPH:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
            for i in range(n):
                fn(i)
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if g is not None:
            g.replay()
        else:
            for i in range(n):
                fn(i)
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) * 1e3 / n)
    return statistics.median(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[33, 48, 64, 85, 96, 128])
    ap.add_argument("--plans", action="store_true", help="also sweep (waves, split) plans")
    ap.add_argument("--proj", nargs="+", default=list(SHAPES))
    ap.add_argument("--graph", action="store_true", help="time graph replays (no host cost)")
    ap.add_argument("--wide-below-33", action="store_true",
                    help="route <= 32-row calls to the wide kernel too (ops.set_wide_min_rows)")
    ap.add_argument("--vs-skinny", action="store_true",
                    help="M <= 32: wide kernel vs the 16-row-tile GEMV (second column)")
    ap.add_argument("--sweep", action="store_true",
                    help="every (waves, split) plan; prints the best per (proj, M)")
    ap.add_argument("--midm-sweep", action="store_true",
                    help="M > 128: every (row-block height, K split) plan of the mid-M kernel")
    ap.add_argument("--tuned", action="store_true",
                    help="library arm on the shipped tuned table, rows padded to its buckets "
                         "(as the engine runs it)")
    ap.add_argument("--model", choices=["8b", "70b"], default="8b")
    ap.add_argument("--fp8", action="store_true",
                    help="fp8 weights: the W8 builds vs the engine's library fp8 chain "
                         "(row-quantised activations + hipBLASLt fp8 GEMM)")
    a = ap.parse_args()
    global GRAPH
    GRAPH = a.graph
    assert ops.native_available(), ops._load_error
    ops.ensure_splitk_workspace("cuda")
    if a.tuned:
        from agentic_traffic_testing_amd import tuning
        print("tuned table:", tuning.load("auto", "llama-3.1-8b" if a.model == "8b"
                                          else "llama-3-70b"), flush=True)
    dt = torch.bfloat16
    hq, hkv, bs, nb = (32 if a.model == "8b" else 64), 8, 16, 512
    shapes = SHAPES if a.model == "8b" else SHAPES_70B
    kc = torch.zeros(nb, hkv, bs, 128, dtype=dt, device="cuda")
    vc = torch.zeros(nb, hkv, 128, bs, dtype=dt, device="cuda")
    cs = ref.rope_cos_sin(128, 8192, 500000.0, None, device="cuda")
    ones = torch.ones(8192, dtype=dt, device="cuda")
    tot = {}
    for proj in a.proj:
        n, k = shapes[proj]
        mb = n * k * (1 if a.fp8 else 2) / 1e6
        ncopy = max(2, int(600 // mb) + 1)
        rowmap = {"qkv": "qkv", "gate_up": "silu"}.get(proj, "plain")
        raw = [(torch.randn(n, k, device="cuda") * 0.02).to(dt) for _ in range(ncopy)]
        scales = [None] * ncopy
        if a.fp8:
            qs = [ops.quantize_fp8(w) for w in raw]
            raw = [q for q, _ in qs]
            scales = [sc for _, sc in qs]
            wps = [ops.preshuffle_fp8(q, rowmap) for q in raw]
        else:
            wps = [ops.preshuffle(w, rowmap) for w in raw]
        for m in a.m:
            x = torch.randn(m, k, device="cuda").to(dt)
            res = torch.zeros(m, n, dtype=dt, device="cuda")
            pos = torch.arange(m, dtype=torch.int32, device="cuda")
            slots = torch.arange(m, dtype=torch.int32, device="cuda")
            q = torch.empty(m, hq, 128, dtype=dt, device="cuda")
            act = torch.empty(m, n // 2, dtype=dt, device="cuda")

            def wide(i, plan=(0, 0), mplan=(0, 0)):
                ops.set_wide_plan(*plan)
                ops.set_midm_plan(*mplan)
                w, sc = wps[i % ncopy], scales[i % ncopy]
                if proj == "qkv":
                    ops.decode_qkv_rope(x, w, 1e-5, pos, slots, cs, kc, vc, hq, hkv, q_out=q,
                                        preshuffled=True, w_scale=sc)
                elif proj == "gate_up":
                    ops.decode_gate_up_silu(x, w, 1e-5, out=act, preshuffled=True, w_scale=sc)
                else:  # as models/llama.py forward_decode calls it
                    ops.linear(x, w, residual=res, preshuffled=True, ksplit=None, proj=proj,
                               waves=ops.decode_waves(proj, True, a.fp8), w_scale=sc)

            ml = m
            if a.tuned and m > 32:
                from agentic_traffic_testing_amd.tuning import bucket_rows
                ml = bucket_rows(m)
            xl = torch.randn(ml, k, device="cuda").to(dt)
            resl = torch.zeros(ml, n, dtype=dt, device="cuda")
            posl = torch.arange(ml, dtype=torch.int32, device="cuda")

            def lib(i):
                w = raw[i % ncopy]
                if a.fp8:  # models/llama.py forward's fp8 chain
                    sc = scales[i % ncopy]
                    if proj == "qkv":
                        xq, xs = ops.quant_rows_fp8(xl, ops.QUANT_NORM, ones[:k], 1e-5)
                        y = ops.gemm_fp8(xq, xs, w, sc, dt)
                        ops.rope_cache(y, posl, posl, cs, kc, vc, hq, hkv, 128)
                    elif proj == "gate_up":
                        xq, xs = ops.quant_rows_fp8(xl, ops.QUANT_NORM, ones[:k], 1e-5)
                        ops.quant_rows_fp8(ops.gemm_fp8(xq, xs, w, sc, dt), ops.QUANT_SILU)
                    else:
                        xq, xs = ops.quant_rows_fp8(xl)
                        ops.gemm_fp8(xq, xs, w, sc, dt)
                    return
                if proj == "qkv":
                    y = torch.nn.functional.linear(ops.rms_norm(xl, ones[:k], 1e-5), w)
                    ops.rope_cache(y, posl, posl, cs, kc, vc, hq, hkv, 128)
                elif proj == "gate_up":
                    ops.silu_and_mul(torch.nn.functional.linear(ops.rms_norm(xl, ones[:k], 1e-5), w))
                else:
                    resl.addmm_(xl, w.t())

            ops.set_wide_min_rows(*((1, 1) if a.wide_below_33 else (17, 12)))
            tw = timeit(wide)
            tl = timeit(lib)
            if a.vs_skinny and m <= 32:
                ops.set_wide_min_rows(33, 33)
                tl = timeit(wide)  # the "library" column holds the 16-row-tile GEMV here
                ops.set_wide_min_rows(1, 1)
                tw = timeit(wide)
            tot.setdefault(m, [0.0, 0.0])
            tot[m][0] += tw
            tot[m][1] += tl
            line = (f"{proj:8s} M={m:4d} | wide {tw:7.1f} us ({mb / tw:5.2f} TB/s) | "
                    f"library {tl:7.1f} us | {tl / tw:5.2f}x")
            if m > 128:
                epi = {"qkv": 2, "gate_up": 3, "o": 1, "down": 1}[proj]
                ntiles = n // 8 // 2 if proj == "gate_up" else n // 16
                line += " | plan bmt %d S %d" % ops.midm_plan(m, ntiles, k, epi)
            if a.midm_sweep and m > 128:
                for xd in (1,):
                    tim = {}
                    splits = (1,) if proj in ("qkv", "gate_up") else (1, 2, 3, 4, 6, 8)
                    for b_ in ops.MIDM_BUILT:
                        for s_ in splits:
                            try:
                                tim[(b_, s_)] = timeit(lambda i, p=(b_, s_): wide(i, mplan=p),
                                                       n=20)
                            except RuntimeError:
                                pass
                    best = min(tim, key=tim.get)
                    line += (f" | xd{xd} best {best[0]}x{best[1]}={tim[best]:.1f} | " +
                             " ".join(f"{k[0]}x{k[1]}={v:.1f}" for k, v in sorted(tim.items())))
            if a.sweep:
                tim = {}
                for w_ in (4, 6, 7, 8):
                    for s_ in (1, 2, 3, 4, 5, 6, 8):
                        try:
                            tim[(w_, s_)] = timeit(lambda i, p=(w_, s_): wide(i, p), n=20)
                        except RuntimeError as e:
                            err = str(e).splitlines()[0]
                assert tim, f"no plan ran: {err}"
                best = min(tim, key=tim.get)
                line += (f" | best {best[0]}x{best[1]}={tim[best]:.1f} | " +
                         " ".join(f"{k[0]}x{k[1]}={v:.1f}" for k, v in sorted(tim.items())))
            if a.plans:
                cells = []
                for w_, s_ in PLANS[proj]:
                    try:
                        cells.append(f"{w_}x{s_}={timeit(lambda i, p=(w_, s_): wide(i, p)):.1f}")
                    except RuntimeError:  # a plan the library does not build at this M
                        cells.append(f"{w_}x{s_}=n/a")
                line += " | plans " + " ".join(cells)
            print(line, flush=True)
        del raw, wps
        torch.cuda.empty_cache()
    for m, (tw, tl) in tot.items():
        print(f"per layer M={m}: wide {tw:7.1f} us, library {tl:7.1f} us ({tl / tw:.2f}x)")


if __name__ == "__main__":
    main()
