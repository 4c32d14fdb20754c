"""CPU backend (BASELINE config 1: agent-a single turn -> CPU model, no GPU).

The reference's ``llm/hf_cpu_server.py`` runs a transformers ``pipeline`` in fp32 on CPU
and serves ``POST /chat|/generate|/completion`` returning only ``{"output"}`` (the prompt
echoed plus a ``temperature=0.7`` sampled completion), without /health or /metrics
(hf_cpu_server.py:34-51, 63-94; SURVEY Appendix B item 7 - a compose swap fails its
healthcheck).  Two modes, both with /health and /metrics:

* ``--hf-compat`` (selected automatically for OPT / GPT-2 ids, e.g. the reference default
  ``facebook/opt-125m``): the model's OWN architecture through transformers
  (serving/hf_compat.py), seeded random-init offline, the reference's sampling and echoed
  output;
* otherwise: the same engine code as the GPU backend on CPU tensors (ops dispatch to the fp32
  reference implementations) with a small Llama-shaped random-init model (``tiny`` preset),
  exposing the full backend API (``{"output", "meta"}``, ``llm_*`` metrics).

Env: ``LLM_MODEL``/``MODEL_NAME`` (default facebook/opt-125m), ``HOST``, ``PORT`` (8000),
``LLM_MAX_TOKENS``, ``LLM_HF_COMPAT=1`` (force the transformers mode).
"""
from __future__ import annotations

import os
import sys

from .serve_llm import apply_config_file, make_parser, run_server


def main(argv=None):
    import asyncio

    p = make_parser()
    p.add_argument("--hf-compat", action="store_true",
                   default=os.environ.get("LLM_HF_COMPAT", "0") == "1",
                   help="serve the model's own architecture through transformers with the "
                        "reference hf_cpu_server contract (automatic for OPT / GPT-2 ids)")
    p.add_argument("--seed", type=int, default=int(os.environ.get("LLM_SEED", "0")),
                   help="random-init seed of the --hf-compat model")
    p.set_defaults(model=os.environ.get("LLM_MODEL") or os.environ.get("MODEL_NAME")
                   or "facebook/opt-125m", host=os.environ.get("HOST", "0.0.0.0"),
                   port=int(os.environ.get("PORT", "8000")), device="cpu", no_graphs=True,
                   max_model_len=int(os.environ.get("LLM_MAX_MODEL_LEN") or 2048))
    args = apply_config_file(p.parse_args(argv))
    from .hf_compat import default_max_tokens, is_hf_family, run

    try:
        if args.hf_compat or is_hf_family(args.model):
            asyncio.run(run(args.model, args.host, args.port, args.seed, default_max_tokens()))
        else:
            os.environ.setdefault("ATTA_CPU_KV_BLOCKS", "512")
            asyncio.run(run_server(args))
    except KeyboardInterrupt:
        print("\n[*] Shutting down CPU backend.")


if __name__ == "__main__":
    sys.exit(main())
