"""The first-8-GPU-lease recipe (scripts/gpu/scale.sh -> scale.py) on the CPU: its
``--device cpu`` twin runs the same sweep with gloo ranks and a tiny model, and every emitted
JSON line must carry the metric / config / n_gpus fields the driver's SCALE run will read
(VERDICT r4 #6)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_scale_recipe_cpu_twin_lines_validate():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["NS"] = "1 2"
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts/gpu/scale.sh"), "--device", "cpu",
                        "--points", "dp", "tp", "70b", "ar"],
                       capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    by = {}
    for o in lines:
        by.setdefault(o["point"], []).append(o)
    assert [o["n_gpus"] for o in by["dp"]] == [1, 2]
    assert [o["n_gpus"] for o in by["tp"]] == [2]
    assert len(by["70b"]) == 1 and len(by["70b-fp8"]) == 1
    from bench import METRIC
    for o in by["dp"] + by["tp"] + by["70b"] + by["70b-fp8"]:
        assert o["check"] == "ok", o
        assert o["config"]["parallelism"] in ("tp1", "dp2", "tp2", "tp8")
        assert o["value"] > 0 and o["n_gpus"] >= 1
    # the metric string names what ran: TP degree and fp8 in it, the BASELINE string only for
    # the headline model at TP=1 (the CPU twin runs the tiny model)
    assert by["tp"][0]["metric"].endswith("tiny-tp8 TP=2")
    assert by["70b"][0]["metric"].endswith("tiny-tp8 TP=8")
    assert by["70b-fp8"][0]["metric"].endswith("tiny-tp8 TP=8 fp8")
    assert "Llama-3-8B TP=1" in METRIC
    ar = by["ar"]
    assert {o["world"] for o in ar} == {2} and all(o["us_per_call"] > 0 for o in ar)
    assert os.path.exists(os.path.join(ROOT, "gpurun_out", "scale.jsonl"))


def test_metric_name_contract():
    from bench import METRIC, metric_name
    assert metric_name("llama-3.1-8b") == METRIC  # the BASELINE.json headline string
    assert metric_name("llama-3.1-8b", 8) == METRIC.replace("TP=1", "TP=8")
    assert metric_name("llama-3-70b", 8, "fp8").endswith("Llama-3-70B TP=8 fp8")
    assert metric_name("llama-3-70b", 1).endswith("Llama-3-70B TP=1")


def test_rccl_rank_parse():
    sys.path.insert(0, os.path.join(ROOT, "scripts", "gpu"))
    import scale
    err = ("NCCL INFO comm 0x55 rank 3 nRanks 8 nNodes 1 localRanks 8 localRank 3 MNNVL 0\n"
           "NCCL INFO ncclCommInitRank comm 0x55 rank 3 nranks 8 cudaDev 3 busId 45000 - Init COMPLETE\n")
    assert scale.rccl_ranks(err) == 8
    assert scale.rccl_ranks("no rccl here") == 0
