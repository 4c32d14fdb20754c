"""Model and engine configuration.

The reference serves ``meta-llama/Llama-3.1-8B-Instruct`` through vLLM with the knobs in
infra/docker-compose.yml:16-27 (dtype float16, max_num_seqs 12, max_num_batched_tokens
8192, gpu_memory_utilization 0.90, max_model_len 4096) and KV blocks of 16 tokens
(llm/serve_llm.py:325).  ``EngineConfig`` keeps those names and defaults; the MI355X
specific additions (tensor/data parallel degree, hipGraph buckets, decode partitioning)
default to values sized for 288 GB of HBM3E per GPU.
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass, field, replace
from pathlib import Path

LLAMA3_ROPE_SCALING = {
    "rope_type": "llama3",
    "factor": 8.0,
    "low_freq_factor": 1.0,
    "high_freq_factor": 4.0,
    "original_max_position_embeddings": 8192,
}


@dataclass(frozen=True)
class ModelConfig:
    name: str = "llama-3.1-8b"
    vocab_size: int = 128256
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_layers: int = 32
    num_heads: int = 32
    num_kv_heads: int = 8
    head_dim: int = 128
    rms_norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    rope_scaling: dict | None = field(default_factory=lambda: dict(LLAMA3_ROPE_SCALING))
    max_position_embeddings: int = 131072
    tie_word_embeddings: bool = False
    bos_token_id: int = 128000
    eos_token_ids: tuple = (128001, 128008, 128009)

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    def num_params(self) -> int:
        h, i, v = self.hidden_size, self.intermediate_size, self.vocab_size
        per_layer = h * (self.q_size + 2 * self.kv_size) + self.q_size * h + 3 * h * i + 2 * h
        emb = v * h * (1 if self.tie_word_embeddings else 2)
        return self.num_layers * per_layer + emb + h

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return self.num_layers * 2 * self.num_kv_heads * self.head_dim * dtype_bytes


MODEL_PRESETS: dict[str, ModelConfig] = {
    "llama-3.1-8b": ModelConfig(),
    "llama-3-8b": ModelConfig(name="llama-3-8b", rope_scaling=None, max_position_embeddings=8192,
                              eos_token_ids=(128001, 128009)),
    "llama-3-70b": ModelConfig(name="llama-3-70b", hidden_size=8192, intermediate_size=28672,
                               num_layers=80, num_heads=64, num_kv_heads=8, rope_scaling=None,
                               max_position_embeddings=8192, eos_token_ids=(128001, 128009)),
    "llama-3.1-70b": ModelConfig(name="llama-3.1-70b", hidden_size=8192, intermediate_size=28672,
                                 num_layers=80, num_heads=64, num_kv_heads=8),
    "llama-3.2-3b": ModelConfig(name="llama-3.2-3b", hidden_size=3072, intermediate_size=8192,
                                num_layers=28, num_heads=24, num_kv_heads=8,
                                tie_word_embeddings=True,
                                rope_scaling=dict(LLAMA3_ROPE_SCALING, factor=32.0)),
    "llama-3.2-1b": ModelConfig(name="llama-3.2-1b", hidden_size=2048, intermediate_size=8192,
                                num_layers=16, num_heads=32, num_kv_heads=8, head_dim=64,
                                tie_word_embeddings=True,
                                rope_scaling=dict(LLAMA3_ROPE_SCALING, factor=32.0)),
    # small shapes for tests / CPU plumbing runs (head_dim 128 like every Llama-3 >= 3B)
    "tiny": ModelConfig(name="tiny", vocab_size=4096, hidden_size=256, intermediate_size=512,
                        num_layers=2, num_heads=4, num_kv_heads=2, max_position_embeddings=4096,
                        bos_token_id=3840, eos_token_ids=(3841, 3849)),
    "small": ModelConfig(name="small", vocab_size=32768, hidden_size=1024, intermediate_size=2816,
                         num_layers=4, num_heads=8, num_kv_heads=2, max_position_embeddings=8192,
                         bos_token_id=32512, eos_token_ids=(32513, 32521)),
    # long-context tests: the "small" shape with a 32k RoPE table (reference .env runs 11k)
    "small-32k": ModelConfig(name="small-32k", vocab_size=32768, hidden_size=1024,
                             intermediate_size=2816, num_layers=4, num_heads=8, num_kv_heads=2,
                             max_position_embeddings=32768, bos_token_id=32512,
                             eos_token_ids=(32513, 32521)),
    # TP rehearsal shape: 8 q heads over 2 KV heads, so TP=4/8 replicate KV heads (kv_rep > 1)
    "tiny-tp8": ModelConfig(name="tiny-tp8", vocab_size=4096, hidden_size=256,
                            intermediate_size=512, num_layers=2, num_heads=8, num_kv_heads=2,
                            max_position_embeddings=4096, bos_token_id=3840,
                            eos_token_ids=(3841, 3849)),
    # 70B attention geometry (GQA 8:1, hidden 8192) with few layers / a small FFN and vocab:
    # the G=8 decode path and 8192-wide GEMVs on one GPU in seconds
    # Llama-3.2-3B geometry (reference infra/.env.example:116): hidden 3072, 24 q / 8 kv heads
    # (GQA G = 3), tied embeddings - 2 layers and a small vocab for GPU tests
    "llama-3b-slice": ModelConfig(name="llama-3b-slice", vocab_size=16384, hidden_size=3072,
                                  intermediate_size=8192, num_layers=2, num_heads=24,
                                  num_kv_heads=8, tie_word_embeddings=True,
                                  rope_scaling=dict(LLAMA3_ROPE_SCALING, factor=32.0),
                                  bos_token_id=16000, eos_token_ids=(16001, 16009)),
    # the Llama-3.1-8B layer geometry (hidden 4096, 32 q / 8 kv heads, FFN 14336) with 2
    # layers and a small vocab: the persistent decode step's shapes on one GPU in seconds
    "llama-8b-slice": ModelConfig(name="llama-8b-slice", vocab_size=16384, hidden_size=4096,
                                  intermediate_size=14336, num_layers=2, num_heads=32,
                                  num_kv_heads=8, max_position_embeddings=16384,
                                  bos_token_id=16000, eos_token_ids=(16001, 16009)),
    # the Llama-3-70B TP=8 per-rank geometry (one KV head and 8 q heads per rank, hidden 8192)
    # with an FFN that stays fused-decode-shaped at TP=2/4/8 (7168 / 8 = 896 = 7 x 128): the
    # one-GPU TP rehearsal of graph-captured decode
    "llama-70b-tp-slice": ModelConfig(name="llama-70b-tp-slice", vocab_size=16384,
                                      hidden_size=8192, intermediate_size=7168, num_layers=2,
                                      num_heads=64, num_kv_heads=8, rope_scaling=None,
                                      max_position_embeddings=16384, bos_token_id=16000,
                                      eos_token_ids=(16001, 16009)),
    # the same per-rank geometry for fp8 weights (BASELINE config 5): the fp8 GEMVs stream K in
    # 256-wide steps (4 waves x 64), so the FFN shard must be a multiple of 256 at TP=8 - the
    # real 70B's 28672 / 8 = 3584 is; this slice's 14336 / 8 = 1792 = 7 x 256 is too
    "llama-70b-tp-slice-fp8": ModelConfig(name="llama-70b-tp-slice-fp8", vocab_size=16384,
                                          hidden_size=8192, intermediate_size=14336,
                                          num_layers=2, num_heads=64, num_kv_heads=8,
                                          rope_scaling=None, max_position_embeddings=16384,
                                          bos_token_id=16000, eos_token_ids=(16001, 16009)),
    "llama-70b-slice": ModelConfig(name="llama-70b-slice", vocab_size=16384, hidden_size=8192,
                                   intermediate_size=3584, num_layers=2, num_heads=64,
                                   num_kv_heads=8, rope_scaling=None,
                                   max_position_embeddings=16384, bos_token_id=16000,
                                   eos_token_ids=(16001, 16009)),
}


def resolve_model(model: str) -> tuple[ModelConfig, str | None]:
    """Map a reference-style model id (``meta-llama/Llama-3.1-8B-Instruct``), a preset name
    or a local HF directory (config.json [+ *.safetensors]) to a ModelConfig.
    Returns (config, weights_dir or None)."""
    p = Path(model)
    if p.is_dir() and (p / "config.json").exists():
        return config_from_hf(p / "config.json"), str(p)
    key = model.lower().split("/")[-1]
    if key in MODEL_PRESETS:
        return MODEL_PRESETS[key], None
    for k in ("3.1-70b", "3.2-3b", "3.2-1b", "3-70b", "3.1-8b", "3-8b"):
        if k in key:
            name = "llama-" + k
            return MODEL_PRESETS[name], None
    if "70b" in key:
        return MODEL_PRESETS["llama-3-70b"], None
    if "opt-125m" in key or "tiny" in key:
        return MODEL_PRESETS["tiny"], None
    return MODEL_PRESETS["llama-3.1-8b"], None


def config_from_hf(path: Path) -> ModelConfig:
    c = json.loads(Path(path).read_text())
    eos = c.get("eos_token_id", 128009)
    eos = tuple(eos) if isinstance(eos, list) else (eos,)
    hd = c.get("head_dim") or c["hidden_size"] // c["num_attention_heads"]
    return ModelConfig(
        name=c.get("_name_or_path", Path(path).parent.name) or "hf-model",
        vocab_size=c["vocab_size"], hidden_size=c["hidden_size"],
        intermediate_size=c["intermediate_size"], num_layers=c["num_hidden_layers"],
        num_heads=c["num_attention_heads"],
        num_kv_heads=c.get("num_key_value_heads", c["num_attention_heads"]), head_dim=hd,
        rms_norm_eps=c.get("rms_norm_eps", 1e-5), rope_theta=c.get("rope_theta", 10000.0),
        rope_scaling=c.get("rope_scaling"),
        max_position_embeddings=c.get("max_position_embeddings", 8192),
        tie_word_embeddings=c.get("tie_word_embeddings", False),
        bos_token_id=c.get("bos_token_id", 128000), eos_token_ids=eos)


def _env_int(name, default):
    v = os.environ.get(name)
    try:
        return int(v) if v not in (None, "") else default
    except ValueError:
        return default


@dataclass
class EngineConfig:
    model: str = "meta-llama/Llama-3.1-8B-Instruct"
    dtype: str = "bfloat16"              # reference default float16; both supported
    # Limit: the flash prefill kernel stages a sequence's whole block-table row in LDS (2048
    # entries = 32k tokens at block_size 16).  max_model_len beyond that sends EVERY prefill
    # to the slower v1 kernel (ops.prefill_impl picks by table width, not by the batch) -
    # raise block_size with it (block_size 32 keeps flash up to 64k).
    max_model_len: int = 4096
    max_num_seqs: int = 12
    max_num_batched_tokens: int = 8192
    gpu_memory_utilization: float = 0.90
    block_size: int = 16                 # VLLM_BLOCK_SIZE default (serve_llm.py:325)
    enable_prefix_caching: bool = True
    tensor_parallel_size: int = 1
    seed: int = 0
    device: str = "cuda"
    # hipGraph capture of decode steps (padded batch buckets)
    use_graphs: bool = True
    graph_batch_sizes: tuple = (1, 2, 4, 8, 16, 32, 64, 128, 256)
    # decode split-K partition size (tokens) for the paged attention kernel
    decode_partition_tokens: int = 256
    # finer split for small decode batches (<= decode_small_batch_max sequences): a partition
    # is one workgroup's K/V stream, and at B <= 8 the attention is bound by per-CU bandwidth
    # x latency (256 tokens = 128 KB per workgroup, ~2.5 us to land: the timeline of
    # scripts/gpu/trace_decode_attention.py), so 128-token partitions put twice the CUs on it;
    # with the one-round-trip merge and partition-bucket graphs this wins in situ (bench
    # 760.5 -> 765.5 tok/s; r1 measured it losing with the old 4-per-round-trip merge).
    # Falls back to decode_partition_tokens when max_model_len needs > 64 partitions.
    decode_partition_tokens_small: int = 128
    # decode hipGraphs per partition bucket (attention grid sized to the step's longest
    # context, not max_model_len); buckets above max_model_len's count are dropped
    graph_parts_buckets: tuple = (1, 2, 4, 6, 8, 12, 16, 24, 32, 48, 64)
    decode_small_batch_max: int = 8
    # optional finest tier: B <= decode_tiny_batch_max splits into 64-token partitions
    # (0 = off, the default: faster in isolation - B = 1 at 0.6-3.5k context 7.3 / 8.8 us vs
    # 8.4 / 10.7 at 128 - but it lost in situ, bench 751.9 vs 756.9 tok/s on one box:
    # profiles/r5_attention_partitions.txt)
    decode_partition_tokens_tiny: int = 64
    decode_tiny_batch_max: int = 0
    # chunked prefill: max prompt tokens of one sequence per step (0 = max_num_batched_tokens)
    long_prefill_token_threshold: int = 0
    # fused native decode path (GEMV kernels) when available
    fused_decode: bool = True
    # burst-aware admission (engine/async_engine.py): requests that announce their fan-out
    # (X-Task-ID + x-fanout headers) are held up to this long for their siblings so the
    # burst shares one prefill; 0 disables.  Requests without the headers are never held.
    burst_window_ms: float = 10.0
    # ... and the window closes early once this long has passed since the burst's latest
    # arrival (a LAN fan-out lands inside ~1 ms; under netem skew early arrivals go ahead)
    burst_gap_ms: float = 4.0
    # prefill projection GEMMs: "hipblaslt", "atta" (hand-written CDNA4 Stream-K GEMM with
    # fused residual-add / SiLU-mul epilogues, bf16 and fp8: ops/csrc/prefill_gemm.hip, for
    # steps of >= prefill_gemm_min_rows tokens) or "auto" (each projection on whichever won
    # the measured A/B at that size: models/llama.py LlamaModel._PG_AUTO - with a shipped
    # tuned table the library wins every shape the workload reaches, round 5)
    prefill_gemm: str = "auto"
    prefill_gemm_min_rows: int = 128
    # prefill steps of <= 32 rows (cached-prompt planning prefills, short chunks) on the fused
    # decode kernels (norm-folded skinny GEMVs, RoPE / KV write / SiLU epilogues)
    small_prefill_fused: bool = True
    # library prefill GEMMs from a TunableOp solution table (rocBLAS / hipBLASLt solution per
    # exact shape, tuned cold on MI355X by scripts/gpu/tune_prefill_gemms.py): "auto" = the
    # table shipped for this GPU (agentic_traffic_testing_amd/tuning/), "" = off, else a path.
    # With a table, prefill steps pad their row count to the table's buckets
    # (tuning.bucket_rows) - padding rows carry slot -1 and are never written to the KV cache
    # or sampled
    gemm_tuning: str = "auto"
    # async look-ahead decode: launch the next decode graph step before waiting for the
    # current one's tokens (llm_engine.LLMEngine.step)
    async_decode: bool = True
    # keep a pre-shuffled copy of the decode-GEMV weights (contiguous 1 KiB wave loads)
    preshuffle_decode_weights: bool = True
    # GPU engine start: run every tuned library GEMM shape once and serve a few throw-away
    # requests of the workload's step shapes (prefix cache dropped after), so no code object
    # (HIP translation unit, rocBLAS / hipBLASLt solution, PyTorch kernel) loads inside a
    # timed request (bench/coldstart.py: first 560-row prefill 1157 ms -> 11.5 ms without)
    startup_warmup: bool = True
    # "" = 16-bit weights; "fp8" = OCP e4m3fn weight-only quantisation with per-row scales
    # (decode: fp8 GEMV kernels; prefill: hipBLASLt fp8 GEMM) - BASELINE config 5
    quantization: str = ""
    num_kv_blocks: int = 0               # 0 = size from gpu_memory_utilization
    load_format: str = "auto"            # auto | dummy (random init) | safetensors
    # tensor parallelism: "auto" = RCCL ("nccl") on GPUs, gloo on CPU; "gloo" forces the
    # host path (e.g. several ranks rehearsing on one GPU); tp_same_device puts every rank
    # on the first device (single-GPU rehearsal of the TP protocol)
    tp_backend: str = "auto"
    tp_same_device: bool = False
    tp_allreduce: str = "auto"           # auto | rccl | ipc (custom one-shot all-reduce)
    # IPC path: the row-parallel o / down decode GEMVs push their partial products straight
    # into the peers' receive slots (all-reduce push fused into the GEMV epilogue)
    tp_fused_push: bool = True
    dist_port: int = 0                   # 0 = pick a free port
    # a TP worker that has not registered on the step channel this long after rank 0
    # created it is reported dead (covers workers that die while loading weights)
    tp_register_timeout_s: float = 900.0

    def replace(self, **kw) -> "EngineConfig":
        return replace(self, **kw)

    def as_dict(self) -> dict:
        return asdict(self)

    @staticmethod
    def from_env(**overrides) -> "EngineConfig":
        """Engine knobs from the reference's env variables (infra/docker-compose.yml:16-27)."""
        cfg = EngineConfig()
        env = os.environ
        kw = {}
        if env.get("LLM_MODEL"):
            kw["model"] = env["LLM_MODEL"]
        if env.get("LLM_DTYPE"):
            kw["dtype"] = env["LLM_DTYPE"]
        n = _env_int("LLM_MAX_NUM_SEQS", -1)
        if n > 0:
            kw["max_num_seqs"] = n
        n = _env_int("LLM_MAX_NUM_BATCHED_TOKENS", -1)
        if n > 0:
            kw["max_num_batched_tokens"] = n
        if env.get("LLM_GPU_MEMORY_UTILIZATION"):
            kw["gpu_memory_utilization"] = float(env["LLM_GPU_MEMORY_UTILIZATION"])
        n = _env_int("LLM_MAX_MODEL_LEN", 0)
        if n > 0:
            kw["max_model_len"] = n
        n = _env_int("VLLM_BLOCK_SIZE", 0)
        if n > 0:
            kw["block_size"] = n
        n = _env_int("LLM_TENSOR_PARALLEL_SIZE", 0)
        if n > 0:
            kw["tensor_parallel_size"] = n
        if env.get("LLM_QUANTIZATION"):
            kw["quantization"] = env["LLM_QUANTIZATION"].strip().lower()
        kw.update({k: v for k, v in overrides.items() if v is not None})
        return cfg.replace(**kw)
