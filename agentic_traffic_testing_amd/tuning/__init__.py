"""Library-GEMM solution tables for the prefill projections (PyTorch TunableOp format).

hipBLASLt's heuristic pick is not the fastest solution at the row counts the agent workload
prefills (~70-row planning calls, ~380-row fan-out bursts, ~3k-row synthesis prompts): the
rocBLAS / hipBLASLt solution search that TunableOp runs finds faster ones per exact shape
(profiles/r4_tunableop_probe.txt).  ``scripts/gpu/tune_prefill_gemms.py`` tunes every
projection of a model at every row bucket below - cold weights, as a real prefill streams
them - and writes ``tunableop_<arch>_<model>.csv`` here; the engine loads the table with
tuning OFF (no tuning stalls while serving) and pads prefill steps to the buckets so every
step's GEMMs hit a tuned shape.
"""
from __future__ import annotations

import os
from pathlib import Path

HERE = Path(__file__).resolve().parent


def bucket_rows(t: int) -> int:
    """Row count a prefill step of t tokens is padded to: multiples of 16 up to 128, of 32 up
    to 512, of 64 up to 1024, of 128 up to 4096, of 256 beyond (at most 1/8 extra rows from
    256 tokens on; below that the GEMMs stream weights and padding rows cost little)."""
    if t <= 0:
        return t
    step = (16 if t <= 128 else 32 if t <= 512 else 64 if t <= 1024 else
            128 if t <= 4096 else 256)
    return (t + step - 1) // step * step


def all_buckets(max_rows: int) -> list[int]:
    out, t = [], 1
    while t <= max_rows:
        b = bucket_rows(t)
        out.append(b)
        t = b + 1
    return out


# presets with the same GEMM shapes share a table (TunableOp keys entries by exact shape; one
# file holds a model's TP=1 shapes and its TP=8 shard shapes)
TABLE_ALIASES = {"llama-3-8b": "llama-3.1-8b", "llama-3.1-70b": "llama-3-70b"}


def table_path(model_name: str, arch: str = "gfx950") -> Path:
    return HERE / f"tunableop_{arch}_{TABLE_ALIASES.get(model_name, model_name)}.csv"


_loaded: str | None = None


def load(spec: str, model_name: str) -> str | None:
    """Enable TunableOp in lookup-only mode with the table ``spec`` names ("auto": the one
    shipped for ``model_name``; "": off).  Returns the loaded path, or None when no table
    applies.  Idempotent per process."""
    global _loaded
    if not spec:
        return None
    path = table_path(model_name) if spec == "auto" else Path(spec)
    if not path.is_file():
        return None
    if _loaded == str(path):
        return _loaded
    import torch

    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(False)          # lookups only: never tune while serving
    tun.record_untuned_enable(False)
    # TunableOp may write its results file at exit: point that at a scratch path, never at
    # the shipped table
    import tempfile

    tun.set_filename(os.path.join(tempfile.gettempdir(), f"atta_tunableop_{os.getpid()}.csv"))
    if not tun.read_file(str(path)):
        tun.enable(False)
        return None
    _loaded = str(path)
    return _loaded
