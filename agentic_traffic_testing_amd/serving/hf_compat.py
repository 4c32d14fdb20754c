"""HF-compatible CPU backend: any transformers causal-LM architecture, the reference's
``llm/hf_cpu_server.py`` contract (BASELINE config 1).

The reference serves ``pipeline("text-generation")`` in fp32 on CPU and answers
``POST /chat|/generate|/completion`` with ``{"output": <prompt + completion>}`` (the
pipeline's ``generated_text`` echoes the prompt), sampling ``temperature=0.7,
do_sample=True`` (hf_cpu_server.py:34-51, 63-94).  This module keeps that contract for every
architecture transformers implements - ``facebook/opt-*`` (the BASELINE config-1 model),
GPT-2, Llama, ... - instead of mapping every id to a Llama preset:

* the model is ``AutoModelForCausalLM.from_config`` of the id's architecture; there is no
  network, so the weights are seeded random-init (``--seed``) unless a local directory with
  ``config.json`` (+ ``*.safetensors``) is given, whose weights are then loaded;
* OPT ids map to their published dimensions (``OPTConfig`` defaults ARE opt-125m);
* text goes through the local ``tokenizer.json`` when the directory has one, else through the
  repo's deterministic synthetic tokenizer sized to the model's vocabulary;
* beyond the reference: ``GET /health|/ready|/live`` and ``/metrics`` (the ``llm_*`` families
  of serving/metrics.py), so a compose healthcheck against it passes (SURVEY Appendix B
  item 7), and a request may ask for ``"temperature": 0`` (greedy) or a ``"seed"``.

Run: ``python -m agentic_traffic_testing_amd.serving.cpu_server --hf-compat`` (OPT / GPT-2 ids
select it automatically).
"""
from __future__ import annotations

import asyncio
import json
import os
import threading
import time
from pathlib import Path

import torch

from ..engine.tokenizer import HFTokenizer, SyntheticTokenizer
from .metrics import CONTENT_TYPE_LATEST, LLMMetrics

# published dimensions of the OPT family (HF config.json of each facebook/opt-* checkpoint)
OPT_SIZES = {
    "125m": {},  # OPTConfig() defaults
    "350m": dict(hidden_size=1024, num_hidden_layers=24, ffn_dim=4096, num_attention_heads=16,
                 word_embed_proj_dim=512, do_layer_norm_before=False),
    "1.3b": dict(hidden_size=2048, num_hidden_layers=24, ffn_dim=8192, num_attention_heads=32,
                 word_embed_proj_dim=2048),
    "2.7b": dict(hidden_size=2560, num_hidden_layers=32, ffn_dim=10240, num_attention_heads=32,
                 word_embed_proj_dim=2560),
}

REFERENCE_TEMPERATURE = 0.7  # hf_cpu_server.py:91


def is_hf_family(model_id: str) -> bool:
    """Ids whose architecture the Llama engine does not implement (served here instead)."""
    k = model_id.lower()
    return any(t in k for t in ("opt-", "/opt", "gpt2", "gpt-2", "distilgpt2"))


def hf_config_for(model_id: str):
    """transformers config of ``model_id``: a local directory's config.json, or the
    published dimensions of a known family (no network)."""
    from transformers import AutoConfig, GPT2Config, OPTConfig

    p = Path(model_id)
    if (p / "config.json").exists():
        return AutoConfig.from_pretrained(str(p))
    k = model_id.lower()
    if "opt" in k:
        size = next((s for s in OPT_SIZES if f"opt-{s}" in k), "125m")
        return OPTConfig(**OPT_SIZES[size])
    if "gpt2" in k or "gpt-2" in k:
        return GPT2Config()
    raise ValueError(f"no offline config for {model_id!r}: pass a local model directory")


class HFCausalLM:
    """A transformers causal LM on CPU in fp32 with the pipeline's text-in / text-out
    generation (prompt echoed in the output)."""

    def __init__(self, model_id: str, seed: int = 0, dtype=torch.float32, threads: int = 0):
        from transformers import AutoModelForCausalLM

        if threads > 0:
            torch.set_num_threads(threads)
        self.model_id = model_id
        self.config = hf_config_for(model_id)
        torch.manual_seed(seed)
        self.model = AutoModelForCausalLM.from_config(self.config).to(dtype).eval()
        p = Path(model_id)
        files = sorted(p.glob("*.safetensors")) if p.is_dir() else []
        if files:
            from safetensors.torch import load_file

            sd = {}
            for f in files:
                sd.update(load_file(str(f)))
            self.model.load_state_dict(sd, strict=False)
        vocab = int(self.config.vocab_size)
        if p.is_dir() and (p / "tokenizer.json").exists():
            self.tok = HFTokenizer(str(p))
            self.bos = getattr(self.config, "bos_token_id", None)
        else:
            self.tok = SyntheticTokenizer(vocab_size=vocab, num_special=min(256, vocab // 4))
            self.bos = self.tok.bos_token_id
        eos = getattr(self.config, "eos_token_id", None)
        self.eos = self.tok.eos_token_id if isinstance(self.tok, SyntheticTokenizer) else eos
        self.max_positions = int(getattr(self.config, "max_position_embeddings", 2048))
        self._lock = threading.Lock()  # one generate at a time (the reference is single-threaded)

    def encode(self, prompt: str) -> list[int]:
        ids = self.tok.encode(prompt)
        return ([self.bos] if self.bos is not None else []) + list(ids)

    def generate_ids(self, ids: list[int], max_new_tokens: int, temperature: float,
                     do_sample: bool, seed: int | None = None) -> list[int]:
        # keep the prompt's head: the position table bounds prompt + completion
        room = max(1, self.max_positions - max_new_tokens)
        ids = ids[:room]
        inp = torch.tensor([ids], dtype=torch.long)
        kw = dict(max_new_tokens=max_new_tokens, pad_token_id=self.eos, eos_token_id=self.eos)
        if do_sample and temperature > 0:
            kw.update(do_sample=True, temperature=temperature, top_k=50, top_p=1.0)
        else:
            kw.update(do_sample=False)
        with self._lock, torch.inference_mode():
            if seed is not None:
                torch.manual_seed(seed)
            out = self.model.generate(inp, attention_mask=torch.ones_like(inp), **kw)
        return out[0, inp.shape[1]:].tolist()

    def generate(self, prompt: str, max_new_tokens: int,
                 temperature: float = REFERENCE_TEMPERATURE, do_sample: bool = True,
                 seed: int | None = None) -> tuple[str, int, int]:
        """(prompt + completion, prompt tokens, completion tokens)."""
        ids = self.encode(prompt)
        new = self.generate_ids(ids, max_new_tokens, temperature, do_sample, seed)
        return prompt + self.tok.decode(new), len(ids), len(new)


def create_app(lm: HFCausalLM, default_max_tokens: int = 512, metrics: LLMMetrics | None = None):
    from aiohttp import web

    metrics = metrics or LLMMetrics(process_collectors=False)
    loop_state = {"inflight": 0}

    async def chat(request: web.Request) -> web.Response:
        t0 = time.perf_counter()
        try:
            data = await request.json()
        except (json.JSONDecodeError, UnicodeDecodeError):
            metrics.requests_total.labels(status="error").inc()
            return web.json_response({"error": "Invalid JSON"}, status=400)
        if not isinstance(data, dict):
            data = {}
        prompt = data.get("prompt") or data.get("input")
        if not isinstance(prompt, str) or not prompt:
            metrics.requests_total.labels(status="error").inc()
            return web.json_response({"error": "Missing 'prompt' field"}, status=400)
        mt = data.get("max_tokens") or data.get("max_new_tokens")
        try:
            mt = int(mt) if mt is not None else default_max_tokens
        except (TypeError, ValueError):
            mt = default_max_tokens
        temp = data.get("temperature", REFERENCE_TEMPERATURE)
        try:
            temp = float(temp)
        except (TypeError, ValueError):
            temp = REFERENCE_TEMPERATURE
        seed = data.get("seed")
        loop_state["inflight"] += 1
        metrics.inflight.set(loop_state["inflight"])
        try:
            text, n_in, n_out = await asyncio.get_running_loop().run_in_executor(
                None, lambda: lm.generate(prompt, max(1, mt), temp, temp > 0,
                                          int(seed) if seed is not None else None))
        except Exception as e:  # noqa: BLE001 - reported to the client as the reference's 500
            metrics.requests_total.labels(status="error").inc()
            return web.json_response({"error": f"{type(e).__name__}: {e}"}, status=500)
        finally:
            loop_state["inflight"] -= 1
            metrics.inflight.set(loop_state["inflight"])
        dt = time.perf_counter() - t0
        metrics.record("ok", dt, 0.0, n_in, n_out)
        return web.json_response({"output": text})

    async def health(_request):
        return web.json_response({"status": "ok", "model": lm.model_id, "backend": "hf-cpu"})

    async def prom(_request):
        return web.Response(body=metrics.exposition(),
                            headers={"Content-Type": CONTENT_TYPE_LATEST})

    app = web.Application()
    for path in ("/chat", "/generate", "/completion"):
        app.router.add_post(path, chat)
    for path in ("/health", "/ready", "/live"):
        app.router.add_get(path, health)
    app.router.add_get("/metrics", prom)
    return app


async def run(model_id: str, host: str, port: int, seed: int = 0,
              default_max_tokens: int = 512) -> None:
    from aiohttp import web

    lm = HFCausalLM(model_id, seed=seed)
    runner = web.AppRunner(create_app(lm, default_max_tokens))
    await runner.setup()
    await web.TCPSite(runner, host, port).start()
    print(f"[*] HF CPU server for {model_id} ({lm.config.model_type}, seeded random-init"
          f" unless a local checkpoint) on http://{host}:{port}", flush=True)
    while True:
        await asyncio.sleep(3600)


def default_max_tokens() -> int:
    return int(os.environ.get("LLM_MAX_TOKENS", "512"))
