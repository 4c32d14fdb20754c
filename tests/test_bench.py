"""bench.py contract on the CPU tier (the driver's SCALE harness runs `bench.py --gpus N`).

* `--gpus 2` launches its own two ranks (torch.distributed.run child, gloo on CPU) and
  reports n_gpus 2 with whole-job tokens/s = the per-rank sum over the slowest wall time;
* `--gpus N` with fewer visible GPUs than N errors out instead of running N=1;
* a mismatch between --gpus and an external WORLD_SIZE is an error;
* `--parallel tp --gpus 2` runs one engine over two ranks.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
SMALL = ["--device", "cpu", "--model", "tiny", "--steps", "1", "--warmup", "0",
         "--max-tokens", "4", "--max-model-len", "1024"]


def _run(args, env=None, timeout=600):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    r = subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True,
                       timeout=timeout, env=e, cwd=ROOT)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, [json.loads(ln) for ln in lines]


def test_bench_gpus2_self_launch_cpu():
    r, out = _run(["--gpus", "2", *SMALL])
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(out) == 1, r.stdout  # ONE line, from rank 0 only
    o = out[0]
    assert o["n_gpus"] == 2 and o["config"]["parallelism"] == "dp2"
    assert len(o["per_rank_tokens_per_s"]) == 2
    assert o["completion_tokens"] == 2 * 7 * 4  # 2 ranks x 7 requests x 4 tokens
    assert o["value"] == pytest.approx(o["completion_tokens"] / (o["ms_per_step"] / 1000.0),
                                       rel=0.02)
    assert o["scaling"] == "weak" and o["higher_is_better"] is True


def test_bench_gpus1_cpu_matches_contract():
    r, out = _run(["--gpus", "1", *SMALL])
    assert r.returncode == 0, r.stderr[-3000:]
    o = out[0]
    assert o["n_gpus"] == 1 and o["config"]["parallelism"] == "tp1"
    for k in ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "vs_baseline",
              "dtype", "data", "config"):
        assert k in o


def test_bench_too_many_gpus_errors():
    r, out = _run(["--gpus", "64", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert out and "error" in out[0] and out[0]["n_gpus"] == 64


def test_bench_world_size_mismatch_errors():
    r, _ = _run(["--gpus", "2", *SMALL], env={"WORLD_SIZE": "1"})
    assert r.returncode != 0 and "does not match WORLD_SIZE" in r.stderr


def test_bench_tp2_cpu():
    r, out = _run(["--gpus", "2", "--parallel", "tp", *SMALL, "--dtype", "float32"])
    assert r.returncode == 0, r.stderr[-3000:]
    o = out[0]
    assert o["n_gpus"] == 2 and o["config"]["parallelism"] == "tp2"
    assert o["scaling"] == "strong" and o["completion_tokens"] == 7 * 4


def test_bench_via_http_cpu():
    """--via http: the fan-out through aiohttp llm-backend + Agent A + 5 Agent B; every LLM
    call of each /task (planning, 5 workers, synthesis) generates exactly max_tokens."""
    r, out = _run([*SMALL, "--via", "http"])
    assert r.returncode == 0, r.stderr[-3000:]
    o = out[-1]
    assert o["via"] == "http" and o["llm_calls"] == 7
    assert o["completion_tokens"] == 7 * 4
    assert o["p50_ttft_s"] is not None and o["p50_ttft_s"] > 0
