#!/usr/bin/env python3
"""First-8-GPU-lease scaling sweep: every point of the scaling curve in one call, one JSON
line per point, each line validated.

Points (GPU):
  dp    bench.py --gpus N (engine replica per GPU, Llama-3.1-8B bf16)   N in $NS (1 2 4 8)
  tp    bench.py --gpus N --parallel tp (8B bf16)                        N in $NS, N > 1
  70b   bench.py --gpus 8 --parallel tp --model llama-3-70b              bf16 and fp8
  ar    scripts/gpu/bench_allreduce.py --world W --distinct --json       IPC one-/two-shot vs
                                                                         RCCL over xGMI
Every bench point runs with NCCL_DEBUG=INFO; the RCCL "nRanks" lines of its stderr are
parsed and the point fails its check unless RCCL reports N ranks (N > 1).  A point whose N
exceeds the visible GPU count prints a ``"skipped"`` line instead of running.  The first
failing point (non-zero exit, time limit, failed check) ends the sweep: nothing else is
started on the GPU after it.

``--device cpu``: the CPU twin (gloo, tiny model, 1 step) of the same sweep, used by
tests/test_scale_recipe.py to validate every emitted line's metric / config / n_gpus fields.

    python scripts/gpu/scale.py                      # GPU, all points
    NS="1 2" python scripts/gpu/scale.py --device cpu --points dp tp
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

from bench import metric_name  # noqa: E402

_NRANKS = re.compile(r"nRanks\s+(\d+)|nranks\s+(\d+)")


def visible_gpus(device: str) -> int:
    if device == "cpu":
        return 64
    import torch  # device_count() does not initialise HIP on this image

    return torch.cuda.device_count()


def rccl_ranks(stderr: str) -> int:
    """Largest rank count any RCCL communicator reported (NCCL_DEBUG=INFO init lines)."""
    best = 0
    for m in _NRANKS.finditer(stderr):
        best = max(best, int(m.group(1) or m.group(2)))
    return best


def plan(points, ns, device):
    """(name, n_gpus, extra bench args, model label, tp degree, quantization) per point."""
    out = []
    for p in points:
        if p == "dp":
            out += [("dp", n, [], "llama-3.1-8b", 1, "") for n in ns]
        elif p == "tp":
            out += [("tp", n, ["--parallel", "tp"], "llama-3.1-8b", n, "") for n in ns if n > 1]
        elif p == "70b":
            for q in ("", "fp8"):
                extra = ["--parallel", "tp", "--model", "llama-3-70b"]
                if q:
                    extra += ["--quantization", q]
                out.append(("70b" + (f"-{q}" if q else ""), 8, extra, "llama-3-70b", 8, q))
        elif p == "ar":
            out += [("ar", n, [], "", n, "") for n in ns if n > 1]
    if device == "cpu":  # the twin: tiny-tp8 (8 q heads, so TP=8 splits), one short step
        twin = []
        for name, n, extra, label, tp, q in out:
            extra = [e for e in extra if e not in ("--model", "llama-3-70b")]
            twin.append((name, n, extra, "tiny-tp8", tp, q))
        out = twin
    return out


def check_line(o: dict, name: str, n: int, label: str, tp: int, q: str, device: str,
               nranks: int) -> list[str]:
    errs = []
    want_metric = metric_name(label, tp if name != "dp" else 1, q)
    if o.get("metric") != want_metric:
        errs.append(f"metric {o.get('metric')!r} != {want_metric!r}")
    if o.get("n_gpus") != n:
        errs.append(f"n_gpus {o.get('n_gpus')} != {n}")
    par = (o.get("config") or {}).get("parallelism")
    want_par = (f"dp{n}" if n > 1 else "tp1") if name == "dp" else f"tp{tp}"
    if par != want_par:
        errs.append(f"parallelism {par!r} != {want_par!r}")
    if not isinstance(o.get("value"), (int, float)) or o["value"] <= 0:
        errs.append(f"value {o.get('value')!r}")
    if o.get("weights") != (q or "bf16") and device != "cpu":
        errs.append(f"weights {o.get('weights')!r}")
    if device != "cpu" and n > 1 and nranks != n:
        errs.append(f"RCCL reported {nranks} ranks, expected {n}")
    return errs


def run_point(name, n, extra, label, tp, q, a, have) -> tuple[bool, list[dict]]:
    base = {"point": name, "n_gpus": n}
    if n > have:
        return True, [{**base, "skipped": f"{have} GPU(s) visible"}]
    env = dict(os.environ, NCCL_DEBUG="INFO", HSA_ENABLE_IPC_MODE_LEGACY="0")
    if name == "ar":
        cmd = [sys.executable, os.path.join(ROOT, "scripts/gpu/bench_allreduce.py"),
               "--world", str(n), "--json"] + (["--distinct"] if a.device == "cuda" else
                                               ["--cpu-twin"])
    else:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
               "--steps", str(a.steps), "--warmup", str(a.warmup), *extra]
        if a.device == "cpu":
            cmd += ["--device", "cpu", "--model", "tiny-tp8", "--max-tokens", "4",
                    "--max-model-len", "1024"]
    t0 = time.monotonic()
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=a.point_timeout,
                           env=env, cwd=ROOT)
    except subprocess.TimeoutExpired:
        return False, [{**base, "error": f"time limit {a.point_timeout}s"}]
    wall = round(time.monotonic() - t0, 1)
    if a.logdir:
        with open(os.path.join(a.logdir, f"scale_{name}_{n}.log"), "w") as f:
            f.write(" ".join(cmd) + "\n" + r.stdout + "\n---- stderr ----\n" + r.stderr)
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return False, [{**base, "error": f"rc {r.returncode}", "wall_s": wall,
                        "stderr_tail": r.stderr[-800:]}]
    if name == "ar":
        return True, [{**base, **ln, "wall_s": wall} for ln in lines]
    o = lines[-1]
    nranks = rccl_ranks(r.stderr)
    errs = check_line(o, name, n, label, tp, q, a.device, nranks)
    o.update(point=name, rccl_nranks=nranks, wall_s=wall, check="ok" if not errs else errs)
    return not errs, [o]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda")
    ap.add_argument("--points", nargs="+", default=["dp", "tp", "70b", "ar"],
                    choices=["dp", "tp", "70b", "ar"])
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--point-timeout", type=int, default=900)
    ap.add_argument("--logdir", default="")
    a = ap.parse_args(argv)
    cpu = a.device == "cpu"
    a.steps = a.steps if a.steps is not None else (1 if cpu else 3)
    a.warmup = a.warmup if a.warmup is not None else (0 if cpu else 1)
    ns = [int(x) for x in os.environ.get("NS", "1 2 4 8").split()]
    if a.logdir:
        os.makedirs(a.logdir, exist_ok=True)
    have = visible_gpus(a.device)
    ok_all = True
    for name, n, extra, label, tp, q in plan(a.points, ns, a.device):
        ok, lines = run_point(name, n, extra, label, tp, q, a, have)
        for ln in lines:
            print(json.dumps(ln), flush=True)
        if not ok:
            ok_all = False
            print(json.dumps({"stop": f"point {name} n={n} failed: the sweep ends here"}),
                  flush=True)
            break
    return 0 if ok_all else 1


if __name__ == "__main__":
    sys.exit(main())
