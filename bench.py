#!/usr/bin/env python3
"""Headline benchmark: llm-backend tokens/s + p50 TTFT under a 5-agent fan-out,
Llama-3-8B (3.1 shape) bf16, TP=1 per engine (BASELINE.json).

One timed *step* = one fan-out episode per rank (agentic_traffic_testing_amd/bench/fanout.py):
planning request -> 5 concurrent Agent-B requests -> final synthesis request, each
generating exactly ``--max-tokens`` (512) tokens with temperature 0.2.

Multi-GPU (one process per GPU):

* ``python bench.py --gpus N`` launches the N ranks ITSELF: it starts
  ``python -m torch.distributed.run --nproc-per-node N`` as a child process (before this
  process touches the GPU; it only counts devices) and exits with the child's status.
  Under an external ``torch.distributed.run`` (WORLD_SIZE set) ``--gpus`` must equal
  WORLD_SIZE.  N larger than the visible GPU count is an error, not a silent N=1 run.
* ``--parallel dp`` (default): every rank is an independent engine replica on its own GPU
  (data-parallel serving, weak scaling); the value is whole-job completion tokens/s (sum
  over ranks / slowest rank's wall time), with the per-rank rates listed too.
* ``--parallel tp``: ONE engine tensor-parallel over the N ranks (rank 0 drives the
  workload; the other ranks replay its steps, parallel/tp_engine.py) - strong scaling.

Weights are seeded random-init of the exact Llama-3.1-8B architecture (``--model
llama-3-70b`` for BASELINE configs 4/5) and prompts are synthetic (no network / gated
checkpoints), which ``data`` states.  ``--device cpu`` runs the same protocol on the CPU
(gloo, tiny models) for the CPU test tier.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "llm-backend tokens/sec + p50 TTFT under 5-agent fan-out, Llama-3-8B TP=1"
DATA = ("synthetic (agent fan-out prompts, synthetic tokenizer, seeded random-init {} "
        "weights)")


def metric_name(label: str, tp: int = 1, quantization: str = "") -> str:
    """The metric string of one run: BASELINE.json's exact METRIC for the headline model at
    TP=1 (a DP replica is a TP=1 engine), otherwise the same template naming the model that
    actually ran, its TP degree and fp8 weights - so a 70B TP=8 record never calls itself
    'Llama-3-8B TP=1'."""
    low = label.lower()
    if "70b" in low:
        fam = "Llama-3-70B"
    elif "8b" in low:
        fam = "Llama-3-8B"
    else:
        fam = label
    if fam == "Llama-3-8B" and tp == 1 and not quantization:
        return METRIC
    q = f" {quantization}" if quantization else ""
    return f"llm-backend tokens/sec + p50 TTFT under 5-agent fan-out, {fam} TP={tp}{q}"


def overrides(items: list[str]) -> dict:
    """--set key=value pairs -> EngineConfig kwargs, typed like the field's default."""
    from dataclasses import fields

    from agentic_traffic_testing_amd.config import EngineConfig

    types = {f.name: type(f.default) for f in fields(EngineConfig)}
    out = {}
    for it in items:
        k, _, v = it.partition("=")
        if k not in types:
            raise SystemExit(f"--set: unknown EngineConfig field {k!r}")
        t = types[k]
        out[k] = (v.lower() in ("1", "true", "yes")) if t is bool else t(v)
    return out


def _window_marker(a):
    """ATTA_WINDOW_MARKERS=1: one tiny stream_read_kernel dispatch at each edge of the timed
    region, so a rocprof kernel trace can be windowed to it (scripts/gpu/summarize_trace.py
    --window stream_read_kernel): init, weight generation and warm-up stay out of the table.
    Outside the timed interval (launched after t_start is read / after elapsed is taken)."""
    if a.device != "cuda" or os.environ.get("ATTA_WINDOW_MARKERS", "0") != "1":
        return
    buf = torch.zeros(4096, dtype=torch.int32, device="cuda")
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    torch.ops.atta.stream_read(buf, sink)
    torch.cuda.synchronize()


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="meta-llama/Llama-3.1-8B-Instruct")
    ap.add_argument("--max-tokens", type=int, default=512)
    ap.add_argument("--fanout", type=int, default=5)
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--max-num-seqs", type=int, default=12)
    ap.add_argument("--max-num-batched-tokens", type=int, default=8192)
    ap.add_argument("--gpu-memory-utilization", type=float, default=0.90)
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: CPU-tier rehearsal of the protocol (gloo, tiny models)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--quantization", default="", choices=["", "fp8"],
                    help="fp8 weight-only quantisation (BASELINE config 5); headline is bf16")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="EngineConfig override for A/B runs (e.g. fuse_attn_oproj=0)")
    ap.add_argument("--parallel", choices=["dp", "tp"], default="dp",
                    help="dp: one engine replica per GPU (default); tp: one engine over all GPUs")
    ap.add_argument("--tp-same-device", action="store_true",
                    help="--parallel tp rehearsal with every rank on cuda:0 (IPC collectives, "
                         "graph-captured decode): the TP protocol on a one-GPU box")
    ap.add_argument("--workload", choices=["agentic_parallel", "agentverse", "proxy"],
                    default="agentic_parallel",
                    help="--via http workload: the /task fan-out (headline), the AgentVerse "
                         "loop (POST /agentverse, config 4) or multi-turn agents through the "
                         "OpenAI-compatible proxy (config 5's MCP-Universe path)")
    ap.add_argument("--arrival-skew-ms", type=float, default=0.0,
                    help="--via http: Agent A sends fan-out worker i's request i * ms late "
                         "(arrival skew, e.g. netem jitter between the agents and the backend)")
    ap.add_argument("--max-tokens-limit", type=int, default=0,
                    help="--via http: clamp every LLM call's max_tokens (0 = off)")
    ap.add_argument("--via", choices=["engine", "http"], default="engine",
                    help="engine: drive the engine in-process (headline); http: the whole "
                         "serving stack - aiohttp llm-backend + Agent A + 5 Agent B over "
                         "127.0.0.1, POST /task agentic_parallel (bench/e2e.py)")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(a) -> int:
    """Start N ranks under torch.distributed.run as a CHILD process and return its status.

    Runs before this process makes any GPU call (device_count() does not initialise HIP on
    this image), so no exec happens from a GPU-initialised process."""
    if a.device == "cuda" and not a.tp_same_device:
        have = torch.cuda.device_count()
        if have < a.gpus:
            print(json.dumps({"metric": METRIC, "error": f"--gpus {a.gpus} requested but only "
                              f"{have} GPU(s) visible", "n_gpus": a.gpus}), flush=True)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", ATTA_BENCH_CHILD="1")
    return subprocess.call(cmd, env=env)


def main(argv=None):
    a = parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(a)
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} does not match WORLD_SIZE {world}")
    if a.parallel == "tp" and world > 1:
        return main_tp(a)
    return main_dp(a, world)


def _cfg(a, device: str, **kw):
    from agentic_traffic_testing_amd.config import EngineConfig

    base = dict(model=a.model, dtype=a.dtype, max_model_len=a.max_model_len,
                max_num_seqs=a.max_num_seqs, max_num_batched_tokens=a.max_num_batched_tokens,
                gpu_memory_utilization=a.gpu_memory_utilization,
                use_graphs=not a.no_graphs and a.device == "cuda", seed=1234, device=device,
                quantization=a.quantization)
    base.update(kw)
    base.update(overrides(a.set))
    return EngineConfig(**base)


def _model_label(a) -> str:
    from agentic_traffic_testing_amd.config import resolve_model

    return resolve_model(a.model)[0].name


def _sync(a):
    if a.device == "cuda":
        torch.cuda.synchronize()


def main_dp(a, world: int):
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    cuda = a.device == "cuda"
    if world > 1:
        import torch.distributed as dist

        if cuda:
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo")
    elif cuda:
        torch.cuda.set_device(0)
    dev = f"cuda:{torch.cuda.current_device()}" if cuda else "cpu"

    from agentic_traffic_testing_amd.bench.fanout import FanoutWorkload
    from agentic_traffic_testing_amd.engine.llm_engine import LLMEngine

    cfg = _cfg(a, dev)
    t0 = time.perf_counter()
    eng = LLMEngine(cfg)
    eng.runner.capture_all(all_parts=True)
    init_s = time.perf_counter() - t0
    wl = FanoutWorkload(eng, fanout=a.fanout, max_tokens=a.max_tokens, seed=rank)

    def log(*x):
        if a.verbose and rank == 0:
            print(*x, file=sys.stderr, flush=True)

    log(f"init {init_s:.1f}s kv_blocks={eng.runner.num_blocks} graphs={sorted(eng.runner.graphs)}")
    if a.via == "http":
        return _finish_http(a, eng, world, rank, dist, init_s, cfg, log)
    for i in range(a.warmup):
        r = wl.run_episode()
        log(f"warmup {i}: {r.completion_tokens / r.seconds:.1f} tok/s, {r.seconds:.2f}s")

    if dist:
        dist.barrier()
    _sync(a)
    _window_marker(a)
    t_start = time.perf_counter()
    results = [wl.run_episode() for _ in range(a.steps)]
    _sync(a)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    _window_marker(a)
    # One untimed COLD episode after the timed region: prefix cache dropped first, so every
    # prompt row is prefilled.  The timed episodes cycle 4 tasks and hit the prefix cache from
    # episode 5 on (only the "(episode N)" suffix is new), so their TTFT is the cached regime;
    # this line reports the uncached one beside it.  Not part of value / ms_per_step.
    cold = None
    if a.steps > 0:
        eng.runner.reset_state()
        cold = wl.run_episode()

    if a.verbose and rank == 0:
        tm = eng.timing
        n = max(1, tm["steps"])
        g = max(1, eng.runner.graph_steps)
        rt = eng.runner.timing
        log(f"host step breakdown over {n} steps: schedule {tm['schedule'] / n * 1e3:.3f} ms, "
            f"execute {tm['execute'] / n * 1e3:.3f} ms, post {tm['post'] / n * 1e3:.3f} ms; "
            f"graph steps {eng.runner.graph_steps}: prep {rt['graph_prep'] / g * 1e3:.3f} ms, "
            f"replay+sync {rt['graph_run'] / g * 1e3:.3f} ms")
    tokens = sum(r.completion_tokens for r in results)
    ttfts = [t for r in results for t in r.ttfts]
    ttft_phases = _phase_table(results)
    cold_phases = _phase_table([cold]) if cold is not None else {}
    cold_ttfts = list(cold.ttfts) if cold is not None else []
    lat = [t for r in results for t in r.latencies]
    per_rank = [round(tokens / elapsed, 2)]
    if dist:
        gathered = [None] * world
        dist.all_gather_object(gathered, (elapsed, tokens, ttfts, lat, cold_ttfts))
        cold_ttfts = [t for g in gathered for t in g[4]]
        elapsed = max(g[0] for g in gathered)
        tokens = sum(g[1] for g in gathered)
        per_rank = [round(g[1] / g[0], 2) for g in gathered]
        ttfts = [t for g in gathered for t in g[2]]
        lat = [t for g in gathered for t in g[3]]
    value = tokens / elapsed
    if rank == 0:
        ms = elapsed / a.steps * 1000.0
        srt = sorted(ttfts)
        p50 = statistics.median(srt) if srt else None
        p95 = srt[min(len(srt) - 1, int(0.95 * len(srt)))] if srt else None
        label = _model_label(a)
        out = {
            "metric": metric_name(label, 1, a.quantization),
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if "bf" in a.dtype else a.dtype,
            "weights": a.quantization or ("bf16" if "bf" in a.dtype else a.dtype),
            "data": DATA.format(label),
            "config": {
                "model": f"{label} (random-init)",
                "global_batch": a.fanout * world,
                "seq_len": a.max_model_len,
                "parallelism": f"dp{world}" if world > 1 else "tp1",
                "max_tokens": a.max_tokens,
                "max_num_seqs": a.max_num_seqs,
                "max_num_batched_tokens": a.max_num_batched_tokens,
                "block_size": cfg.block_size,
                "temperature": 0.2,
                "hipgraphs": cfg.use_graphs,
                "device": a.device,
            },
            "per_rank_tokens_per_s": per_rank,
            "p50_ttft_s": round(p50, 4) if p50 is not None else None,
            "p95_ttft_s": round(p95, 4) if p95 is not None else None,
            "p50_latency_s": round(statistics.median(lat), 3) if lat else None,
            "ttft_by_phase": ttft_phases,
            "p50_ttft_uncached_s": (round(statistics.median(cold_ttfts), 4)
                                    if cold_ttfts else None),
            "ttft_by_phase_uncached": cold_phases,
            "requests_per_step_per_gpu": 2 + a.fanout,
            "completion_tokens": int(tokens),
            "init_s": round(init_s, 1),
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def _phase_table(results) -> dict:
    """TTFT by phase of the episode: rows actually prefilled (prompt - prefix-cache hits) and
    the median TTFT of the phase's requests."""
    by_phase = {}
    for r in results:
        for name, pt, ct, tt in r.phases:
            d = by_phase.setdefault(name, {"rows": [], "ttft": []})
            d["rows"].append(pt - ct)
            d["ttft"].extend(tt)
    return {k: {"prefill_rows": int(statistics.median(v["rows"])),
                "p50_ttft_ms": round(statistics.median(v["ttft"]) * 1e3, 2)}
            for k, v in by_phase.items()}


def _finish_http(a, eng, world, rank, dist, init_s, cfg, log):
    """--via http: the fan-out through the real serving stack on every rank."""
    from agentic_traffic_testing_amd.bench.e2e import run_e2e

    if dist:
        dist.barrier()
    _sync(a)
    r = run_e2e(eng, a.steps, a.warmup, fanout=a.fanout, max_tokens=a.max_tokens, log=log,
                workload=a.workload, max_tokens_limit=a.max_tokens_limit,
                arrival_skew_ms=a.arrival_skew_ms)
    _sync(a)
    elapsed, tokens = r["seconds"], r["tokens"]
    per_rank = [round(r["tokens_per_s"], 2)]
    p50, p95 = r["p50_ttft_s"], r["p95_ttft_s"]
    if dist:
        gathered = [None] * world
        dist.all_gather_object(gathered, (elapsed, tokens, p50, p95))
        elapsed = max(g[0] for g in gathered)
        tokens = sum(g[1] for g in gathered)
        per_rank = [round(g[1] / g[0], 2) for g in gathered]
        p50 = statistics.median(g[2] for g in gathered if g[2] is not None)
        p95 = max(g[3] for g in gathered if g[3] is not None)
    if rank == 0:
        label = _model_label(a)
        print(json.dumps({
            "metric": metric_name(label, 1, a.quantization), "value": round(tokens / elapsed, 2),
            "unit": "tokens/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1000.0, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if "bf" in a.dtype else a.dtype,
            "weights": a.quantization or ("bf16" if "bf" in a.dtype else a.dtype),
            "data": DATA.format(label), "via": "http", "workload": a.workload,
            "config": {"model": f"{label} (random-init)", "global_batch": a.fanout * world,
                       "seq_len": a.max_model_len,
                       "parallelism": f"dp{world}" if world > 1 else "tp1",
                       "max_tokens": a.max_tokens, "hipgraphs": cfg.use_graphs,
                       "stack": "aiohttp llm-backend + agent-a + 5 agent-b (127.0.0.1)",
                       "device": a.device},
            "per_rank_tokens_per_s": per_rank,
            "p50_ttft_s": round(p50, 4) if p50 is not None else None,
            "p95_ttft_s": round(p95, 4) if p95 is not None else None,
            "llm_calls": r["calls"], "llm_calls_per_workflow": r["calls_per_workflow"],
            "peak_inflight": r["peak_inflight"], "bursts_coalesced": r["bursts_coalesced"],
            "ttft_breakdown": r.get("ttft_breakdown"), "arrival_skew_ms": a.arrival_skew_ms,
            "burst_window_ms": cfg.burst_window_ms, "burst_gap_ms": cfg.burst_gap_ms,
            "completion_tokens": int(tokens),
            "per_task_s": r["per_task_s"], "init_s": round(init_s, 1)}), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def main_tp(a):
    """Tensor-parallel bench: ranks > 0 serve rank 0's steps until it stops them."""
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ.get("RANK", "0"))
    dev = "cuda" if a.device == "cuda" else "cpu"
    kw = dict(tp_same_device=True, tp_allreduce="ipc") if a.tp_same_device else {}
    cfg = _cfg(a, dev, tensor_parallel_size=world, **kw)
    port = int(os.environ.get("MASTER_PORT", "29511"))
    if rank > 0:
        from agentic_traffic_testing_amd.parallel.tp_engine import run_worker

        run_worker(cfg, rank, world, port)
        return 0
    from agentic_traffic_testing_amd.bench.fanout import FanoutWorkload
    from agentic_traffic_testing_amd.parallel.tp_engine import TPEngine

    t0 = time.perf_counter()
    eng = TPEngine(cfg, external=True)
    init_s = time.perf_counter() - t0
    try:
        wl = FanoutWorkload(eng, fanout=a.fanout, max_tokens=a.max_tokens, seed=0)
        for _ in range(a.warmup):
            wl.run_episode()
        eng.runner.barrier()
        t_start = time.perf_counter()
        results = [wl.run_episode() for _ in range(a.steps)]
        eng.runner.barrier()
        elapsed = time.perf_counter() - t_start
    except BaseException:
        eng.shutdown()
        raise
    tokens = sum(r.completion_tokens for r in results)
    ttfts = sorted(t for r in results for t in r.ttfts)
    label = _model_label(a)
    out = {
        "metric": metric_name(label, world, a.quantization), "value": round(tokens / elapsed, 2),
        "unit": "tokens/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1000.0, 2), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "bf16" if "bf" in a.dtype else a.dtype,
        "weights": a.quantization or ("bf16" if "bf" in a.dtype else a.dtype),
        "data": DATA.format(label),
        "config": {"model": f"{label} (random-init)", "global_batch": a.fanout,
                   "seq_len": a.max_model_len, "parallelism": f"tp{world}",
                   "max_tokens": a.max_tokens, "hipgraphs": cfg.use_graphs,
                   "tp_allreduce": cfg.tp_allreduce, "device": a.device,
                   "tp_same_device": cfg.tp_same_device},
        "graph_steps": eng.runner.graph_steps, "steps_total": eng.runner.steps,
        "p50_ttft_s": round(statistics.median(ttfts), 4) if ttfts else None,
        "p95_ttft_s": round(ttfts[min(len(ttfts) - 1, int(0.95 * len(ttfts)))], 4)
        if ttfts else None,
        "completion_tokens": int(tokens), "init_s": round(init_s, 1),
    }
    print(json.dumps(out), flush=True)
    eng.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
