"""Llama-3 decoder (8B / 70B / 3.2 shapes) over the atta op layer.

This is the model vLLM executes inside ``AsyncLLMEngine`` for the reference
(llm/serve_llm.py:362-378; model id from infra/docker-compose.yml:26).  MI355X design:

* weights are stored pre-fused: ``qkv`` [(Hq+2Hkv)*D, H], ``gate_up`` [2I, H] so each layer
  runs 4 GEMMs (hipBLASLt via F.linear for prefill-sized M; the decode path can swap in
  the fused GEMV kernels of ``ops``), and every elementwise step is a hand-written kernel:
  fused residual-add+RMSNorm, RoPE+paged-KV write, paged attention (prefill and decode
  variants), SiLU-mul, sampler;
* tensor parallelism is Megatron-style: qkv / gate_up column-parallel, o / down row-parallel
  with one all-reduce each (``parallel.comm``); the embedding is replicated and the LM head
  is vocab-parallel: the fused decode sampler reduces each shard to one packed key per row
  and an int64 MAX all-reduce picks the winner (prefill all-gathers the [B, V/tp] logits);
* weights are either seeded random-init (benchmarks: no network, gated checkpoints) or
  loaded from HF safetensors.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass
from pathlib import Path

import torch
import torch.nn.functional as F

from .. import ops
from ..config import ModelConfig
from ..ops import reference as ref

DTYPES = {"bfloat16": torch.bfloat16, "bf16": torch.bfloat16, "float16": torch.float16,
          "fp16": torch.float16, "half": torch.float16, "auto": torch.bfloat16,
          "float32": torch.float32, "fp32": torch.float32}  # fp32: CPU reference runs only


def torch_dtype(name: str) -> torch.dtype:
    return DTYPES.get(str(name).replace("torch.", ""), torch.bfloat16)


@dataclass
class AttnMeta:
    """Per-step attention metadata (all device tensors, built by the model runner)."""
    positions: torch.Tensor       # int32 [T]
    slot_mapping: torch.Tensor    # int32 [T]
    block_tables: torch.Tensor    # int32 [S, W]
    seq_kvlen: torch.Tensor       # int32 [S]
    seq_qstart: torch.Tensor      # int32 [S+1]
    tile_seq: torch.Tensor        # int32 [tiles]   (prefill sequences)
    tile_qoff: torch.Tensor       # int32 [tiles]
    logits_idx: torch.Tensor      # int64 [S]
    num_decode: int               # sequences [0, num_decode) have exactly one query token
    num_tiles: int


@dataclass
class LayerWeights:
    input_norm: torch.Tensor
    qkv: torch.Tensor
    o: torch.Tensor
    post_norm: torch.Tensor
    gate_up: torch.Tensor
    down: torch.Tensor
    # decode copies in the GEMV's pre-shuffled layout (ops.preshuffle); None = use the
    # row-major weights above
    qkv_ps: torch.Tensor | None = None
    o_ps: torch.Tensor | None = None
    gate_up_ps: torch.Tensor | None = None
    down_ps: torch.Tensor | None = None
    # fp8 weight-only quantisation (GPU): the projections above are uint8 e4m3fn bytes and
    # these are their fp32 per-output-row scales
    qkv_s: torch.Tensor | None = None
    o_s: torch.Tensor | None = None
    gate_up_s: torch.Tensor | None = None
    down_s: torch.Tensor | None = None


class LlamaModel:
    def __init__(self, cfg: ModelConfig, dtype=torch.bfloat16, device="cuda", tp_rank: int = 0,
                 tp_size: int = 1, tp_group=None, quantization: str = ""):
        # tp_group: parallel.comm.TPComm (required when tp_size > 1)
        # quantization: "" (16-bit weights) | "fp8" (OCP e4m3fn weights, per-row scales; on the
        # CPU reference path the dequantised values are stored instead)
        if quantization not in ("", "fp8"):
            raise ValueError(f"unsupported quantization {quantization!r}")
        self.quant = quantization
        # prefill projections: "hipblaslt" (torch / hipBLASLt GEMMs) or "atta" (the
        # hand-written CDNA4 GEMM, ops/csrc/prefill_gemm.hip) for >= prefill_gemm_min_rows rows
        self.prefill_gemm = "auto"
        self.prefill_gemm_min_rows = 128
        # prefill steps of <= 32 rows on the fused decode kernels (EngineConfig.small_prefill_fused)
        self.small_prefill_fused = True
        # the runner's fused-decode switch (EngineConfig.fused_decode): off also turns the
        # fused kernels off for small prefill steps
        self.fused_decode = True
        self.cfg = cfg
        self.dtype = dtype
        self.device = torch.device(device)
        self.tp_rank, self.tp_size, self.tp_group = tp_rank, tp_size, tp_group
        if cfg.num_heads % tp_size:
            raise ValueError(f"num_heads {cfg.num_heads} not divisible by tp {tp_size}")
        self.n_heads = cfg.num_heads // tp_size
        # KV heads are split when possible, replicated when tp > num_kv_heads
        self.kv_rep = max(1, tp_size // cfg.num_kv_heads)
        self.n_kv_heads = max(1, cfg.num_kv_heads // tp_size)
        self.head_dim = cfg.head_dim
        self.inter = cfg.intermediate_size // tp_size
        if cfg.intermediate_size % tp_size or cfg.vocab_size % tp_size:
            raise ValueError("intermediate/vocab not divisible by tp")
        self.vocab_shard = cfg.vocab_size // tp_size
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.layers: list[LayerWeights] = []
        self.lm_head_ps = None
        self.embed = None
        self.norm = None
        self.lm_head = None
        self.cos_sin = ref.rope_cos_sin(cfg.head_dim, min(cfg.max_position_embeddings, 1 << 17),
                                        cfg.rope_theta, cfg.rope_scaling, device=self.device)
        self.g = self.n_heads // self.n_kv_heads
        if self.head_dim != 128 and self.device.type == "cuda":
            raise ValueError("HIP attention kernels require head_dim 128")

    # ---------------------------------------------------------------------------------
    @property
    def qkv_width(self) -> int:
        return (self.n_heads + 2 * self.n_kv_heads) * self.head_dim

    def init_random(self, seed: int = 0, std: float = 0.02):
        """Seeded random-init weights of the full architecture (each rank draws its shard
        from the full-model generator stream so TP=N reproduces TP=1 exactly)."""
        cfg, dev, dt = self.cfg, self.device, self.dtype
        gen_dev = dev if dev.type == "cuda" else torch.device("cpu")
        g = torch.Generator(device=gen_dev)

        def rnd(shape, tag: int, scale=std):
            g.manual_seed(seed * 1000003 + tag)
            return (torch.randn(shape, generator=g, device=gen_dev, dtype=torch.float32)
                    * scale).to(dt).to(dev)

        H, D = cfg.hidden_size, cfg.head_dim
        self.embed = rnd((cfg.vocab_size, H), 1, 1.0)

        def norm_w(tag):  # non-trivial norm weights so the folding is exercised
            return (1.0 + rnd((H,), tag, 0.1).float()).to(dt)

        self.norm = norm_w(3)
        lm = self.embed if cfg.tie_word_embeddings else rnd((cfg.vocab_size, H), 2)
        self.lm_head = self._shard_rows(lm, self.vocab_shard).contiguous()
        self.layers = []
        for i in range(cfg.num_layers):
            base = 100 + i * 10
            wq = rnd((cfg.q_size, H), base + 0)
            wk = rnd((cfg.kv_size, H), base + 1)
            wv = rnd((cfg.kv_size, H), base + 2)
            wo = rnd((H, cfg.q_size), base + 3)
            wg = rnd((cfg.intermediate_size, H), base + 4)
            wu = rnd((cfg.intermediate_size, H), base + 5)
            wd = rnd((H, cfg.intermediate_size), base + 6) / math.sqrt(2 * cfg.num_layers) * 4
            self.layers.append(self._make_layer(wq, wk, wv, wo, wg, wu, wd, norm_w(base + 7),
                                                norm_w(base + 8)))
            del wq, wk, wv, wo, wg, wu, wd
        self._fold_final_norm()
        return self

    def _shard_rows(self, w: torch.Tensor, rows: int) -> torch.Tensor:
        if self.tp_size == 1:
            return w
        return w[self.tp_rank * rows:(self.tp_rank + 1) * rows]

    def _shard_cols(self, w: torch.Tensor, cols: int) -> torch.Tensor:
        if self.tp_size == 1:
            return w
        return w[:, self.tp_rank * cols:(self.tp_rank + 1) * cols]

    def _make_layer(self, wq, wk, wv, wo, wg, wu, wd, n_in, n_post) -> LayerWeights:
        D = self.head_dim
        q = self._shard_rows(wq, self.n_heads * D)
        kv_rank = self.tp_rank // self.kv_rep
        if self.tp_size == 1:
            k, v = wk, wv
        else:
            k = wk[kv_rank * self.n_kv_heads * D:(kv_rank + 1) * self.n_kv_heads * D]
            v = wv[kv_rank * self.n_kv_heads * D:(kv_rank + 1) * self.n_kv_heads * D]
        qkv = torch.cat([q, k, v], 0).contiguous()
        o = self._shard_cols(wo, self.n_heads * D).contiguous()
        gu = torch.cat([self._shard_rows(wg, self.inter), self._shard_rows(wu, self.inter)],
                       0).contiguous()
        down = self._shard_cols(wd, self.inter).contiguous()
        # Fold the RMSNorm weights into the following projections (x*w) W^T = x (W diag(w))^T:
        # the decode kernels then only need the per-row rms, and the prefill path normalises
        # with a unit weight.  Both paths see identical folded weights.
        qkv = (qkv.float() * n_in.float()[None, :]).to(qkv.dtype).contiguous()
        gu = (gu.float() * n_post.float()[None, :]).to(gu.dtype).contiguous()
        ones = self._ones(n_in)
        if self.quant == "fp8":
            # row-parallel shards (o, down: a K slice of every row) quantise with the FULL
            # row's scale, so TP=N fp8 weights equal TP=1's bit for bit
            full = self.tp_size > 1
            amax = (wo.float().abs().amax(1) if full else None,
                    wd.float().abs().amax(1) if full else None)
            return self._quantize_layer(ones, qkv, o, gu, down, amax)
        return LayerWeights(ones, qkv, o, ones, gu, down)

    def _quantize_layer(self, ones, qkv, o, gu, down, amax=(None, None)) -> LayerWeights:
        """fp8 weight-only quantisation of the four projections (after norm folding)."""
        qs = [ops.quantize_fp8(qkv), ops.quantize_fp8(o, amax[0]), ops.quantize_fp8(gu),
              ops.quantize_fp8(down, amax[1])]
        if self.device.type != "cuda":  # CPU reference: the values fp8 can represent
            deq = [ops.dequantize_fp8(q, sc, self.dtype) for q, sc in qs]
            return LayerWeights(ones, deq[0], deq[1], ones, deq[2], deq[3])
        return LayerWeights(ones, qs[0][0], qs[1][0], ones, qs[2][0], qs[3][0],
                            qkv_s=qs[0][1], o_s=qs[1][1], gate_up_s=qs[2][1], down_s=qs[3][1])

    def _ones(self, like):
        if getattr(self, "_ones_t", None) is None or self._ones_t.shape != like.shape:
            self._ones_t = torch.ones_like(like)
        return self._ones_t

    def _fold_final_norm(self):
        self.lm_head = (self.lm_head.float() * self.norm.float()[None, :]).to(
            self.lm_head.dtype).contiguous()
        self.norm = self._ones(self.norm)

    def load_safetensors(self, path: str):
        """Load HF Llama weights (model*.safetensors) and shard for this TP rank."""
        from safetensors import safe_open

        p = Path(path)
        files = sorted(p.glob("*.safetensors"))
        if not files:
            raise FileNotFoundError(f"no safetensors in {path}")
        index = {}
        for f in files:
            with safe_open(str(f), framework="pt") as sf:
                for k in sf.keys():
                    index[k] = f

        def get(name):
            with safe_open(str(index[name]), framework="pt") as sf:
                return sf.get_tensor(name).to(self.dtype).to(self.device)

        cfg = self.cfg
        self.embed = get("model.embed_tokens.weight")
        self.norm = get("model.norm.weight")
        lm = self.embed if cfg.tie_word_embeddings or "lm_head.weight" not in index else get(
            "lm_head.weight")
        self.lm_head = self._shard_rows(lm, self.vocab_shard).contiguous()
        self.layers = []
        for i in range(cfg.num_layers):
            pre = f"model.layers.{i}."
            self.layers.append(self._make_layer(
                get(pre + "self_attn.q_proj.weight"), get(pre + "self_attn.k_proj.weight"),
                get(pre + "self_attn.v_proj.weight"), get(pre + "self_attn.o_proj.weight"),
                get(pre + "mlp.gate_proj.weight"), get(pre + "mlp.up_proj.weight"),
                get(pre + "mlp.down_proj.weight"), get(pre + "input_layernorm.weight"),
                get(pre + "post_attention_layernorm.weight")))
        self._fold_final_norm()
        return self

    def prepare_decode_weights(self):
        """Build pre-shuffled copies of every decode-GEMV weight (row-major originals stay
        for the hipBLASLt prefill GEMMs): each wave load of the decode kernels then reads one
        contiguous 1 KiB instead of 16 rows x 64 B.  Costs one extra copy of the weights,
        which 288 GB of HBM affords (16 GB for Llama-3-8B)."""
        if self.device.type != "cuda":
            return self
        for L in self.layers:
            if L.qkv_s is not None:  # fp8: 16-row x 64-col blocks of bytes
                L.qkv_ps = ops.preshuffle_fp8(L.qkv, "qkv")
                L.o_ps = ops.preshuffle_fp8(L.o)
                L.gate_up_ps = ops.preshuffle_fp8(L.gate_up, "silu")
                L.down_ps = ops.preshuffle_fp8(L.down)
                continue
            L.qkv_ps = ops.preshuffle(L.qkv, "qkv")
            L.o_ps = ops.preshuffle(L.o)
            L.gate_up_ps = ops.preshuffle(L.gate_up, "silu")
            L.down_ps = ops.preshuffle(L.down)
        self.lm_head_ps = ops.preshuffle(self.lm_head)
        torch.cuda.synchronize(self.device)
        return self

    def decode_copy_bytes(self) -> int:
        """Bytes ``prepare_decode_weights`` adds (one copy of every decode GEMV weight)."""
        ts = [self.lm_head] + [w for l in self.layers for w in (l.qkv, l.o, l.gate_up, l.down)]
        return sum(t.numel() * t.element_size() for t in ts)

    # ---------------------------------------------------------------------------------
    def weight_bytes(self) -> int:
        """Bytes of the weights one forward streams (row-major copies, scales included)."""
        ts = [self.embed, self.norm, self.lm_head]
        for l in self.layers:
            ts += [l.input_norm, l.qkv, l.o, l.post_norm, l.gate_up, l.down, l.qkv_s, l.o_s,
                   l.gate_up_s, l.down_s]
        return sum(t.numel() * t.element_size() for t in ts if t is not None)

    @staticmethod
    def _proj(x, w, scale, residual=None):
        """Prefill / generic projection: fp8 weights go through the fp8 GEMM path."""
        if scale is None:
            return ops.linear(x, w, residual=residual)
        y = ops.linear_fp8(x, w, scale)
        if residual is not None:
            return residual.add_(y)
        return y

    def _all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        if self.tp_size > 1:
            self.tp_group.all_reduce(x)
        return x

    def forward(self, input_ids: torch.Tensor, md: AttnMeta, k_caches, v_caches,
                part_out=None, part_lse=None, num_parts: int = 1, part_tokens: int = 256,
                prev_tokens=None, feed_prev=None, rows: torch.Tensor | None = None):
        """Returns the final normed hidden state rows [T, H] - or only ``rows`` (int64 row
        indices, e.g. each sequence's last token) when given: the final norm then runs on
        those rows alone."""
        cfg = self.cfg
        eps = cfg.rms_norm_eps
        # the residual stream IS the embedding output: every row-parallel projection adds its
        # product into it inside the GEMM epilogue (hipBLASLt beta=1 C-matrix epilogue, or the
        # skinny GEMV's RESADD) - no separate add / copy passes over [T, hidden]
        residual = ops.embed(self.embed, input_ids, prev_tokens, feed_prev)
        T = residual.shape[0]
        nq, nkv, D = self.n_heads, self.n_kv_heads, self.head_dim
        # fp8 weights on the GPU: every projection is ONE fp8 GEMM with row-wise scales whose
        # activation operand comes quantised out of the norm / SiLU-mul kernel that produced it
        fp8 = self.quant == "fp8" and self.device.type == "cuda"
        dt = residual.dtype
        pending = None  # fp8: the previous down_proj output, added by the next norm kernel
        # small steps (<= 32 rows: cached-prompt planning prefills, short chunks) run the fused
        # decode kernels - RMSNorm folded into the skinny GEMVs over the pre-shuffled weights,
        # RoPE + KV write in the QKV epilogue, SiLU-mul in gate_up - around the prefill
        # attention: 5 launches per layer at weight-stream speed instead of ~9 with the
        # row-major skinny / library GEMMs (17 rows: 168 -> ~80 us of GEMMs per layer,
        # profiles/r4_small_prefill_fused.txt)
        # fp8 steps of 129.. rows in the MIDM_FP8_ROWS range run every projection on the
        # mid-M kernel's W8 builds (all or nothing: the library fp8 chain defers each down
        # product into the next layer's norm-quant kernel, which a fused qkv cannot take)
        small = self.small_prefill_ok(T) or (fp8 and self.midm_fp8_ok(T))
        # 129..640-row steps (uncached burst / planning prefills): per projection, the mid-M
        # kernel (ops/csrc/midm.h, fused epilogues) where it beats the tuned library GEMM +
        # separate norm / RoPE / SiLU kernels, the library elsewhere (midm_route)
        mid = {} if (small or fp8) else self.midm_route(T)
        for li, L in enumerate(self.layers):
            ps = L.qkv_ps is not None
            if small or mid.get("qkv"):
                q = ops.decode_qkv_rope(residual, L.qkv_ps if ps else L.qkv, eps, md.positions,
                                        md.slot_mapping, self.cos_sin, k_caches[li],
                                        v_caches[li], nq, nkv, preshuffled=ps, w_scale=L.qkv_s)
            else:
                if fp8:
                    if pending is None:
                        xq, xs = ops.quant_rows_fp8(residual, ops.QUANT_NORM, L.input_norm, eps)
                    else:
                        xq, xs = ops.quant_rows_fp8(pending, ops.QUANT_ADDNORM, L.input_norm,
                                                    eps, residual)
                    qkv = self._gemm8(xq, xs, L.qkv, L.qkv_s, dt, "qkv")
                elif self._pg(T, L.qkv, proj="qkv"):
                    qkv = ops.prefill_gemm(ops.rms_norm(residual, L.input_norm, eps), L.qkv)
                else:
                    qkv = self._proj(ops.rms_norm(residual, L.input_norm, eps), L.qkv, L.qkv_s)
                q = ops.rope_cache(qkv, md.positions, md.slot_mapping, self.cos_sin,
                                   k_caches[li], v_caches[li], nq, nkv, D)
            attn = torch.empty_like(q)
            if md.num_decode > 0:
                ops.attention_decode(q, k_caches[li], v_caches[li], md.block_tables,
                                     md.seq_kvlen, md.seq_qstart, self.scale, part_out, part_lse,
                                     num_parts, part_tokens, out=attn, num_seqs=md.num_decode)
            if md.num_tiles > 0:
                ops.attention_prefill(q, k_caches[li], v_caches[li], md.block_tables,
                                      md.seq_kvlen, md.seq_qstart, md.tile_seq, md.tile_qoff,
                                      self.scale, out=attn)
            if fp8 and not small:
                aq, as_ = ops.quant_rows_fp8(attn.view(T, nq * D))
                y = self._all_reduce(self._gemm8(aq, as_, L.o, L.o_s, dt, "o"))
                xq, xs = ops.quant_rows_fp8(y, ops.QUANT_ADDNORM, L.post_norm, eps, residual)
                if self._pg(T, xq, L.gate_up, mode=ops.GEMM_SILU, proj="gate_up"):
                    # SiLU-mul fused into the gate_up GEMM epilogue: [T, I] out, plain quant
                    act = ops.prefill_gemm(xq, L.gate_up, ops.GEMM_SILU, xs=xs, ws=L.gate_up_s)
                    aq, as_ = ops.quant_rows_fp8(act)
                else:
                    gu = ops.gemm_fp8(xq, xs, L.gate_up, L.gate_up_s, dt)
                    aq, as_ = ops.quant_rows_fp8(gu, ops.QUANT_SILU)
                pending = self._all_reduce(self._gemm8(aq, as_, L.down, L.down_s, dt, "down"))
                continue
            if small or mid.get("o"):
                self._row_parallel(attn.view(T, nq * D), L, "o", residual)
            else:
                self._proj_residual(attn.view(T, nq * D), L.o, L.o_s, residual, "o")
            if small and fp8 and T > self._fp8_gate_up_max():
                # fp8 gate_up past its crossover: the library fp8 GEMM on row-quantised
                # activations (norm fused into the quantiser), bf16 SiLU-mul for the fused down
                xq, xs = ops.quant_rows_fp8(residual, ops.QUANT_NORM, L.post_norm, eps)
                a = ops.silu_and_mul(self._gemm8(xq, xs, L.gate_up, L.gate_up_s, dt, "gate_up"))
            elif small or mid.get("gate_up"):
                a = ops.decode_gate_up_silu(residual, L.gate_up_ps if ps else L.gate_up, eps,
                                            preshuffled=ps, w_scale=L.gate_up_s)
            else:
                x = ops.rms_norm(residual, L.post_norm, eps)
                if self._pg(T, L.gate_up, mode=ops.GEMM_SILU, proj="gate_up"):
                    a = ops.prefill_gemm(x, L.gate_up, ops.GEMM_SILU)
                else:
                    gu = self._proj(x, L.gate_up, L.gate_up_s)
                    a = ops.silu_and_mul(gu)
            if small or mid.get("down"):
                self._row_parallel(a, L, "down", residual)
            else:
                self._proj_residual(a, L.down, L.down_s, residual, "down")
        if rows is not None:
            residual = residual.index_select(0, rows)
            pending = None if pending is None else pending.index_select(0, rows)
        if pending is not None:
            return ops.fused_add_rms_norm(pending, residual, self.norm, eps)
        return ops.rms_norm(residual, self.norm, eps)

    # "auto" routing of the prefill projections: (weight dtype, mode) -> the smallest row count
    # from which the hand-written GEMM beat hipBLASLt in the cold-weight A/B on the 8B shapes.
    # Round 4 re-measured against the library as the engine now runs it
    # (profiles/r4_prefill_gemm_largem_ab.txt): bf16 on the tuned table (gemm_tuning) wins every
    # projection at 2048-4096 rows (the hand-written gate_up+SiLU 0.84-0.88x), so bf16 routes
    # here only when no tuned table is loaded (round 3: 1.06-1.10x over the untuned heuristic at
    # 2600); fp8 gate_up+SiLU 1.08x at 3200, parity at 2048, 0.82-0.92x below; fp8 down
    # 0.89-0.93x (was routed from 2048 in round 3).
    # Against the shipped tuned tables the hand-written prefill GEMM wins nowhere that the
    # workload reaches (round 5, profiles/r5_prefill_gemm_vs_tuned.txt: fp8 gate_up+SiLU
    # 0.88-0.95x at 2560-3200 rows, bf16 down split-K 0.59-1.03x at 448-1152), so with a table
    # loaded nothing is routed to it; without one (models with no shipped table) it keeps the
    # shapes where it beat the untuned library (r3 / r4)
    _PG_AUTO: dict = {}
    _PG_AUTO_UNTUNED = {(torch.bfloat16, "gate_up"): 2048, (torch.uint8, "gate_up"): 2560}
    gemm_tuned = False  # set by the model runner when a tuned library table is loaded
    # row ranges where the split-K schedule (co-resident K slices of the few 256 x 256 tiles,
    # parallel reduction) beat the UNTUNED hipBLASLt: bf16 down+residual 1.12-1.15x at M 512 /
    # 1024, parity at 400 (profiles/r3_prefill_gemm_ab_bf16_splitk.txt); not used with a table
    _PG_SPLITK = {(torch.bfloat16, "down"): (448, 1152)}

    def _pg_splitk(self, T: int, w: torch.Tensor, proj: str) -> bool:
        if (self.prefill_gemm != "auto" or self.device.type != "cuda" or self.tp_size > 1
                or self.gemm_tuned):
            return False
        lo, hi = self._PG_SPLITK.get((w.dtype, proj), (1, 0))
        return lo <= T <= hi

    def _pg(self, T: int, *ops_, mode: int = 0, proj: str = "") -> bool:
        """Route this prefill projection to the hand-written CDNA4 GEMM (ops.prefill_gemm):
        ``prefill_gemm == "atta"`` (from ``prefill_gemm_min_rows`` rows) or ``"auto"`` (the
        measured winners, _PG_AUTO), for shapes it takes.  Called as _pg(T, w) for bf16
        (activation shape implied) or _pg(T, xq, w, mode)."""
        if self.device.type != "cuda":
            return False
        w = ops_[-1]
        if self.prefill_gemm == "auto":
            m = self._PG_AUTO.get((w.dtype, proj))
            if m is None and not self.gemm_tuned:
                m = self._PG_AUTO_UNTUNED.get((w.dtype, proj))
            if m is None or T < m:
                return False
        elif self.prefill_gemm != "atta" or T < self.prefill_gemm_min_rows:
            return False
        if len(ops_) == 1:
            w = ops_[0]
            x = torch.empty_strided((T, w.shape[1]), (w.shape[1], 1), dtype=w.dtype, device="meta")
            return ops.prefill_gemm_ok(x, w, mode)
        return ops.prefill_gemm_ok(ops_[0], ops_[1], mode)

    def _gemm8(self, xq, xs, w, ws, dt, proj=""):
        """fp8 prefill projection: the hand-written fp8 GEMM when routed there, else the
        hipBLASLt row-scaled GEMM."""
        if self._pg(xq.shape[0], xq, w, proj=proj):
            return ops.prefill_gemm(xq, w, xs=xs, ws=ws)
        return ops.gemm_fp8(xq, xs, w, ws, dt)

    def _proj_residual(self, x, w, scale, residual, proj=""):
        """residual += x @ w.T (row-parallel projection; TP: all-reduced partial sums)."""
        if (scale is None and self._pg_splitk(x.shape[0], w, proj)
                and ops.prefill_gemm_ok(x, w, ops.GEMM_RESADD)):
            # split-K needs its T * S workgroups co-resident: TP = 1 only (one process per GPU)
            return ops.prefill_gemm(x, w, ops.GEMM_RESADD, residual=residual, schedule="splitk")
        if scale is None and self._pg(x.shape[0], x, w, mode=ops.GEMM_RESADD, proj=proj):
            if self.tp_size > 1:
                return self.tp_group.all_reduce_residual(ops.prefill_gemm(x, w), residual)
            return ops.prefill_gemm(x, w, ops.GEMM_RESADD, residual=residual)
        if self.tp_size > 1:
            # residual += sum over ranks, the add fused into the IPC reduction's epilogue
            return self.tp_group.all_reduce_residual(self._proj(x, w, scale), residual)
        return self._proj(x, w, scale, residual=residual)

    # Per-projection row ranges where the mid-M kernel (fused epilogues included) beat the tuned
    # library GEMM plus its separate norm / RoPE / SiLU kernels at the 8B shapes, cold weights,
    # library rows padded to the tuning buckets as the engine runs them
    # (profiles/r6_midm_vs_tuned.txt): qkv + RoPE 1.05-1.48x at 129-640 rows, down + residual
    # 1.03-1.41x at 129-640, o + residual 1.05-1.17x at 129-188 and 1.06-1.12x at 448-640;
    # gate_up + SiLU loses everywhere (0.59-0.93x: the kernel streams ~52 GB/s per CU at ~35 %
    # MFMA, the library's 256-wide tiles run ~41 %).
    MIDM_ROUTES = {"qkv": ((129, 640),), "o": ((129, 188), (448, 640)), "gate_up": (),
                   "down": ((129, 640),)}

    def midm_route(self, T: int) -> dict:
        """{projection: True} for the projections of a T-row step that run the mid-M kernel
        (empty when the step cannot: TP, fp8, no pre-shuffled weights, rows past
        ops.MIDM_MAX_M)."""
        if (T <= 128 or T > ops.fused_max_rows(True, False) or self.quant == "fp8"
                or self.tp_size != 1 or not self.fused_decode or not self.small_prefill_fused
                or not self.decode_fusable(min(T, 128)) or not self.layers
                or self.layers[0].qkv_ps is None):
            return {}
        return {p: any(lo <= T <= hi for lo, hi in r) for p, r in self.MIDM_ROUTES.items()}

    # fp8 (weight-only) steps of these rows run the whole layer on the mid-M kernel's W8
    # builds instead of the row-quantised library fp8 GEMMs (ATTA_MIDM_FP8_ROWS="lo-hi").  Off
    # by default: the library's fp8 MFMA GEMMs win from 274 rows on at the 8B shapes (bench
    # fp8 uncached planning 274 rows 5.68 vs 7.47 ms, burst 392 rows 6.42 vs 9.35 ms,
    # profiles/r6_midm_fp8_negative.txt) - the W8 builds run bf16 MFMAs at ~35 % busy
    _fp8_rows = os.environ.get("ATTA_MIDM_FP8_ROWS", "0")
    MIDM_FP8_ROWS = ((0, -1) if _fp8_rows in ("", "0") else
                     tuple(int(v) for v in _fp8_rows.split("-")))

    # fp8 weights, TP = 1: most rows of a fused-path step whose gate_up + SiLU still runs the
    # wide kernel's W8 build, by hidden size; past it the library fp8 GEMM wins (cold weights,
    # bench_wide --fp8 --tuned, profiles/r6_wide_fp8.txt: 8B 38.4 vs 47.4 us at 75 rows, 50.9
    # vs 47.4 at 128; 70B 106 vs 117 at 33 rows, 123 vs 118 at 64).  qkv / o / down keep the
    # W8 builds to 128 rows (1.14-1.9x at <= 96 rows, 0.93-0.97x at 128 on the 70B shapes)
    FP8_GATE_UP_WIDE_MAX = {4096: 112, 8192: 48}
    # and the whole fused step: 70B fp8 prefill 33 / 76 / 112 / 128 rows 15.4 / 21.4 / 23.8 /
    # 24.3 ms fused vs 20.6 / 22.4 / 23.2 / 23.3 on the library chain
    # (profiles/r6_70b_fp8_planning_prefill.txt)
    FP8_FUSED_MAX_ROWS = {8192: 96}

    def _fp8_fused_max(self) -> int:
        if self.tp_size > 1:
            return 128
        return self.FP8_FUSED_MAX_ROWS.get(self.cfg.hidden_size, 128)

    def _fp8_gate_up_max(self) -> int:
        if self.tp_size > 1:
            return 128  # the TP shards' library GEMMs are launch-bound: not measured past it
        return self.FP8_GATE_UP_WIDE_MAX.get(self.cfg.hidden_size, 128)

    def midm_fp8_ok(self, T: int) -> bool:
        """Does an fp8 step of T > 128 rows run every projection on the mid-M W8 builds?"""
        lo, hi = self.MIDM_FP8_ROWS
        return (self.quant == "fp8" and 128 < T and lo <= T <= hi
                and T <= ops.fused_max_rows(True, True) and self.tp_size == 1
                and self.fused_decode and self.small_prefill_fused
                and self.device.type == "cuda" and self.decode_fusable(T))

    def small_prefill_ok(self, T: int) -> bool:
        """Does a (prefill or mixed) step of T rows run on the fused decode kernels - RMSNorm
        folded into the pre-shuffled skinny GEMVs, RoPE + KV write in the QKV epilogue, SiLU-mul
        in gate_up?  The one predicate for forward() and the runner's row padding (ADVICE r4:
        steps that take the library path are padded to its tuned buckets; fused_decode=False
        turns the fused kernels off here too).  Up to 128 rows, 16-bit or fp8 weights, any TP
        degree (the row-parallel sums go through _row_parallel); past 128 rows every
        projection is routed on its own (midm_route)."""
        if self.quant == "fp8":
            if T > self._fp8_fused_max() or not (self.layers and self.layers[0].qkv_ps is not None):
                return False
        return (self.small_prefill_fused and self.fused_decode and self.device.type == "cuda"
                and T <= 128 and self.decode_fusable(T))

    def decode_fusable(self, num_tokens: int) -> bool:
        """Can a step of this many rows run the fused weight-streaming kernels?  <= 32 rows:
        the 16-row-tile GEMVs (any layout); 33..128 rows: the wide small-M kernel over the
        pre-shuffled 16-bit or fp8 weights (any TP degree: past the fused push's 32 rows the
        row-parallel sums take the IPC / RCCL all-reduce); 129..ops.MIDM_MAX_M rows: the mid-M
        kernel (16-bit weights, TP = 1)."""
        # 16-bit GEMVs: K % 128 (4 waves x 32); fp8 GEMVs: K % 256 (4 waves x 64)
        step = 256 if self.quant == "fp8" else 128
        dims = (self.device.type == "cuda" and self.cfg.hidden_size % step == 0
                and self.inter % step == 0 and (self.n_heads * self.head_dim) % step == 0)
        if not dims or num_tokens < 1:
            return False
        if num_tokens <= ops.SKINNY_MAX_M:
            return True
        lim = ops.fused_max_rows(True, self.quant == "fp8")
        if self.tp_size > 1:
            lim = min(lim, 128)  # the mid-M routes are measured at TP = 1 shapes only
        return (num_tokens <= lim and bool(self.layers) and self.layers[0].qkv_ps is not None
                and self.lm_head_ps is not None)

    def hidden_fusable(self) -> bool:
        """The LM-head GEMV streams K = hidden in 128-wide (16-bit) wave steps."""
        return self.device.type == "cuda" and self.cfg.hidden_size % 128 == 0

    def forward_decode(self, input_ids: torch.Tensor, md: AttnMeta, k_caches, v_caches, ws: dict,
                       temperature, seeds, steps, prev_tokens=None,
                       feed_prev=None, top_p=None, top_k=None) -> torch.Tensor:
        """Fused decode step (every sequence has one query token); returns sampled ids.

        Per layer: [RMSNorm+QKV+RoPE+KV-write] -> [paged attention, in-kernel split-K
        combine] -> [o_proj + residual add] -> [RMSNorm+gate_up+SiLU*up] ->
        [down_proj + residual add]; then [final RMSNorm + LM head + sampler].  5 kernels per
        layer instead of ~10, no normalised activations or logits ever hit HBM.  With
        ``top_p`` / ``top_k`` (per-row device tensors) the step ends in final RMSNorm + LM head
        + the top-k / top-p sampler kernel instead (logits materialised)."""
        eps = self.cfg.rms_norm_eps
        nq, nkv = self.n_heads, self.n_kv_heads
        B = input_ids.shape[0]
        residual = ops.embed(self.embed, input_ids, prev_tokens, feed_prev)
        q = ws["q"][:B]
        attn = ws["attn"][:B]
        act = ws["act"][:B]
        for li, L in enumerate(self.layers):
            ps = L.qkv_ps is not None
            if L.qkv_s is not None and not ps:
                raise RuntimeError("fp8 decode needs prepare_decode_weights()")
            wq = L.qkv_ps if ps else L.qkv
            ops.decode_qkv_rope(residual, wq, eps, md.positions, md.slot_mapping, self.cos_sin,
                                k_caches[li], v_caches[li], nq, nkv, q_out=q, preshuffled=ps,
                                w_scale=L.qkv_s)
            ops.attention_decode_v2(q, k_caches[li], v_caches[li], md.block_tables,
                                    md.seq_kvlen, md.seq_qstart, self.scale, ws["part_out"],
                                    ws["part_lse"], ws["counters"], ws["max_parts"],
                                    ws["part_tokens"], out=attn, num_seqs=B)
            self._row_parallel(attn.view(B, nq * self.head_dim), L, "o", residual)
            ops.decode_gate_up_silu(residual, L.gate_up_ps if ps else L.gate_up, eps, out=act,
                                    preshuffled=ps, w_scale=L.gate_up_s)
            self._row_parallel(act, L, "down", residual)
        if top_p is not None:
            logits = self.compute_logits(ops.rms_norm(residual, self.norm, eps))
            return ops.sample_topkp(logits, temperature, top_p, top_k, seeds, steps,
                                    out=ws["tokens"][:B])
        return self.sample_rows(residual, eps, temperature, seeds, steps, ws)

    def _row_parallel(self, x: torch.Tensor, L, proj: str, residual: torch.Tensor) -> None:
        """residual += x @ W.T for the row-parallel o / down projection on the fused kernels
        (16-row-tile GEMV, wide or mid-M kernel; fp8 weights with their row scales).  TP: the
        GEMV epilogue pushes the partial product into the peers' IPC slots and one receive
        kernel adds the rank-order sum into the residual (X1 / X2, <= 32 rows), else the
        product goes through the all-reduce whose epilogue adds it (IPC one- / two-shot, or
        RCCL)."""
        ps = L.qkv_ps is not None
        w = getattr(L, proj + "_ps") if ps else getattr(L, proj)
        scale = getattr(L, proj + "_s")
        waves = ops.decode_waves(proj, ps, scale is not None)
        if self.tp_size == 1:
            ops.linear(x, w, residual=residual, waves=waves, preshuffled=ps, w_scale=scale,
                       ksplit=None, proj=proj)
        elif self.tp_group.push_ok(x.shape[0], w.shape[0]):
            ops.linear_push_reduce(x, w, residual, self.tp_group.ipc, waves=waves,
                                   preshuffled=ps, w_scale=scale, proj=proj)
        else:
            self.tp_group.all_reduce_residual(
                ops.linear(x, w, waves=waves, preshuffled=ps, w_scale=scale, ksplit=None,
                           proj=proj), residual)

    def sample_rows(self, x, eps, temperature, seeds, steps, ws) -> torch.Tensor:
        """[final RMSNorm (eps > 0) +] LM head + sampler for <= 32 rows without materialising
        logits; tokens land in ws["tokens"][:B] on every rank (an async look-ahead step embeds
        them from there).  Used by the fused decode step and for the last-token rows of
        prefill steps (their rows are already normalised: eps = 0)."""
        B = x.shape[0]
        lm_ps = self.lm_head_ps is not None
        lm = self.lm_head_ps if lm_ps else self.lm_head
        if self.tp_size == 1:
            return ops.decode_lm_head_sample(x, lm, eps, temperature, seeds, steps, ws["keys"],
                                             tokens=ws["tokens"][:B], preshuffled=lm_ps)
        # TP: each rank samples its vocab shard down to one packed key per row (global ids,
        # so the Gumbel noise equals TP=1's); one int64 MAX all-reduce picks the winner
        keys = ops.decode_lm_head_sample(x, lm, eps, temperature, seeds, steps, ws["keys"],
                                         tokens=ws["tp_keys"][:B], finalize="key",
                                         vocab_offset=self.tp_rank * self.vocab_shard,
                                         preshuffled=lm_ps)
        toks = ws["tokens"][:B]
        self.tp_group.all_reduce_max(keys, tokens=toks)  # IPC: one kernel, tokens included
        return toks

    def compute_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        logits = ops.linear(hidden, self.lm_head)
        if self.tp_size > 1:
            logits = self.tp_group.all_gather_last(logits)
        return logits


def save_config_json(cfg: ModelConfig, path: str):
    Path(path).write_text(json.dumps(cfg.__dict__, indent=2, default=list))
