"""CPU plumbing backend (BASELINE config 1: agent-a single turn -> CPU model, no GPU).

The reference's ``llm/hf_cpu_server.py`` runs a transformers ``pipeline`` in fp32 on CPU
and serves ``POST /chat|/generate|/completion`` returning only ``{"output"}``, without
/health or /metrics (hf_cpu_server.py:63-94; SURVEY Appendix B item 7 - a compose swap
fails its healthcheck).  This server runs the same engine code as the GPU backend on CPU
tensors (ops dispatch to the fp32 reference implementations) with a small Llama-shaped
random-init model (``facebook/opt-125m`` and other ids map to the ``tiny`` preset), and
exposes the full backend API including /health and /metrics, so it is a drop-in
replacement for the GPU backend in compose files and tests.

Env: ``LLM_MODEL``/``MODEL_NAME`` (default facebook/opt-125m), ``HOST``, ``PORT`` (8000),
``LLM_MAX_TOKENS``.
"""
from __future__ import annotations

import os
import sys

from .serve_llm import apply_config_file, make_parser, run_server


def main(argv=None):
    import asyncio

    p = make_parser()
    p.set_defaults(model=os.environ.get("LLM_MODEL") or os.environ.get("MODEL_NAME")
                   or "facebook/opt-125m", host=os.environ.get("HOST", "0.0.0.0"),
                   port=int(os.environ.get("PORT", "8000")), device="cpu", no_graphs=True,
                   max_model_len=int(os.environ.get("LLM_MAX_MODEL_LEN") or 2048))
    args = apply_config_file(p.parse_args(argv))
    os.environ.setdefault("ATTA_CPU_KV_BLOCKS", "512")
    try:
        asyncio.run(run_server(args))
    except KeyboardInterrupt:
        print("\n[*] Shutting down CPU backend.")


if __name__ == "__main__":
    sys.exit(main())
