"""Op layer: CDNA4 HIP kernels (``torch.ops.atta``) with device-strict dispatch.

* GPU tensors always run the hand-written HIP kernels from ``_atta_kernels.so``.  If the
  library is missing or fails to load, GPU calls raise ``NativeKernelsUnavailable`` -
  there is no silent eager fallback on a GPU.
* CPU tensors run ``reference.py`` (the same math in fp32 PyTorch) so the whole engine can
  be exercised in the CPU test tier.
"""
from __future__ import annotations

import os
from pathlib import Path

import torch

from . import reference as ref

_LIB = Path(__file__).resolve().parent / "_atta_kernels.so"
_loaded = False
_load_error: str | None = None


class NativeKernelsUnavailable(RuntimeError):
    pass


def library_build_hash(path: Path = _LIB) -> str | None:
    """Source hash embedded in a built kernel library (ops/build.py), or None."""
    import ctypes

    try:
        fn = ctypes.CDLL(str(path)).atta_build_hash
    except (OSError, AttributeError):
        return None
    fn.restype = ctypes.c_char_p
    return fn().decode()


def _lib_embeds(digest: str) -> bool:
    try:
        return digest.encode() in _LIB.read_bytes()
    except OSError:
        return False


def load_native(build_if_missing: bool = True) -> bool:
    """Load the HIP kernel library.  With ``build_if_missing`` the library is (re)built
    in-tree when missing or when its sources changed (content-hash stamps); without it a
    library whose embedded source hash does not match the sources is refused."""
    global _loaded, _load_error
    if _loaded:
        return True
    try:
        from . import build

        want = build.kernel_source_hash()
        # a library that embeds the current source hash is used as is (checked on the file
        # bytes, without loading it): the object files and their stamps need not exist - a
        # gpurun snapshot ships the .so only, and N ranks importing at once must not rebuild
        if build_if_missing and not _lib_embeds(want):
            build.build_kernels()  # serialised across processes by a file lock
        got = library_build_hash()
        if got != want:
            raise RuntimeError(f"stale kernel library {_LIB}: built from sources {got}, "
                               f"tree has {want}")
        torch.ops.load_library(str(_LIB))
        _loaded = True
        _load_error = None
        torch.ops.atta.set_flash_waves(FLASH_WAVES)  # the host tiles follow this setting
        torch.ops.atta.set_splitk_half(SPLITK_HALF)
        torch.ops.atta.set_flash_split_blocks(FLASH_SPLIT_BLOCKS)
        if WIDE_MAX_M <= SKINNY_MAX_M:  # wide kernel off: no <= 32-row call may take it
            torch.ops.atta.set_wide_min_rows(33, 33)
    except Exception as e:  # pragma: no cover - depends on environment
        _load_error = f"{type(e).__name__}: {e}"
    return _loaded


def native_available() -> bool:
    return load_native(build_if_missing=os.environ.get("ATTA_NO_BUILD", "0") != "1")


def _native():
    if not native_available():
        raise NativeKernelsUnavailable(
            f"atta HIP kernels not loadable from {_LIB}: {_load_error}. "
            "Run `python -m agentic_traffic_testing_amd.ops.build`.")
    return torch.ops.atta


# ---------------------------------------------------------------------------------------
def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor | None = None):
    if not x.is_cuda:
        r = ref.rms_norm(x, w, eps)
        if out is not None:
            out.copy_(r)
            return out
        return r
    out = torch.empty_like(x) if out is None else out
    _native().rms_norm(out, x, w, eps)
    return out


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                       out: torch.Tensor | None = None):
    """residual <- x + residual (in place); returns rmsnorm(residual) * w."""
    if not x.is_cuda:
        n, r = ref.fused_add_rms_norm(x, residual, w, eps)
        residual.copy_(r)
        if out is not None:
            out.copy_(n)
            return out
        return n
    out = torch.empty_like(x) if out is None else out
    _native().fused_add_rms_norm(out, residual, x, w, eps)
    return out


def silu_and_mul(x: torch.Tensor, out: torch.Tensor | None = None):
    if not x.is_cuda:
        r = ref.silu_and_mul(x)
        if out is not None:
            out.copy_(r)
            return out
        return r
    if out is None:
        out = torch.empty(x.shape[0], x.shape[1] // 2, dtype=x.dtype, device=x.device)
    _native().silu_and_mul(out, x)
    return out


def embed(table: torch.Tensor, ids: torch.Tensor, prev: torch.Tensor | None = None,
          feed_prev: torch.Tensor | None = None, out: torch.Tensor | None = None):
    """Token-embedding gather.  With the int32 device flag ``feed_prev[0]`` set, row r takes
    token ``prev[r]`` (the previous step's device samples) instead of ``ids[r]`` - how an
    async-decode look-ahead step gets inputs the host has not seen yet."""
    T = ids.shape[0]
    if not table.is_cuda:
        src = ids
        if prev is not None and feed_prev is not None and int(feed_prev[0]) != 0:
            src = prev[:T]
        r = torch.nn.functional.embedding(src.long().clamp(0, table.shape[0] - 1), table)
        if out is not None:
            out.copy_(r)
            return out
        return r
    if out is None:
        out = torch.empty(T, table.shape[1], dtype=table.dtype, device=table.device)
    if ids.dtype != torch.int32:
        ids = ids.to(torch.int32)
    if prev is None or feed_prev is None:
        prev = feed_prev = None
    _native().embed(out, table, ids.contiguous(), prev, feed_prev)
    return out


# Bounds-checked debug mode: ATTA_DEBUG_CHECKS=1 validates every paged-KV
# launch's block-table / slot / length arguments against the cache before the kernel runs
# (the kernels themselves index unchecked: a bad page id there is an out-of-bounds HBM access
# that can fault the GPU).  Checks synchronise with the device, so they are skipped inside
# hipGraph capture; combine with HIP_LAUNCH_BLOCKING=1 to pin a fault to its launch.
DEBUG_CHECKS = os.environ.get("ATTA_DEBUG_CHECKS", "0") == "1"


class PagedArgsError(ValueError):
    pass


def _capturing(t: torch.Tensor) -> bool:
    return t.is_cuda and torch.cuda.is_current_stream_capturing()


def check_paged_args(k_cache, block_tables, seq_kvlen, num_seqs: int = -1, what: str = ""):
    """Every block-table entry a sequence's kvlen reaches names a cache page, and the table
    row is long enough.  Raises PagedArgsError (debug mode only; no-op while capturing)."""
    if not DEBUG_CHECKS or _capturing(block_tables):
        return
    n = seq_kvlen.shape[0] if num_seqs < 0 else num_seqs
    nb, bs = k_cache.shape[0], k_cache.shape[2]
    bt = block_tables[:n].long()
    kv = seq_kvlen[:n].long()
    need = (kv + bs - 1) // bs
    if n and int(need.max()) > bt.shape[1]:
        raise PagedArgsError(f"{what}: kvlen {int(kv.max())} needs {int(need.max())} pages, "
                             f"block table has {bt.shape[1]} columns")
    used = torch.arange(bt.shape[1], device=bt.device)[None, :] < need[:, None]
    bad = used & ((bt < 0) | (bt >= nb))
    if bool(bad.any()):
        s, c = (int(i) for i in bad.nonzero()[0])
        raise PagedArgsError(f"{what}: sequence {s} page slot {c} = {int(bt[s, c])} outside "
                             f"the cache's {nb} pages")


def check_slots(k_cache, slots, what: str = ""):
    """KV-write slots are -1 (skip) or inside the cache.  Debug mode only."""
    if not DEBUG_CHECKS or _capturing(slots) or slots.numel() == 0:
        return
    cap = k_cache.shape[0] * k_cache.shape[2]
    sl = slots.long()
    if bool(((sl < -1) | (sl >= cap)).any()):
        raise PagedArgsError(f"{what}: slot ids outside [-1, {cap}): "
                             f"min {int(sl.min())}, max {int(sl.max())}")


def rope_cache(qkv, positions, slot_mapping, cos_sin, k_cache, v_cache, n_q_heads, n_kv_heads,
               head_dim, q_out: torch.Tensor | None = None):
    """Rotate q/k, write k/v to the paged cache; returns q [T, Hq, D]."""
    check_slots(k_cache, slot_mapping, "rope_cache")
    if not qkv.is_cuda:
        q = ref.rope_cache(qkv, positions, slot_mapping, cos_sin, k_cache, v_cache, n_q_heads,
                           n_kv_heads, head_dim)
        if q_out is not None:
            q_out.copy_(q)
            return q_out
        return q
    if q_out is None:
        q_out = torch.empty(qkv.shape[0], n_q_heads, head_dim, dtype=qkv.dtype, device=qkv.device)
    _native().rope_cache(q_out, k_cache, v_cache, qkv, positions, slot_mapping, cos_sin,
                         n_q_heads, n_kv_heads, head_dim)
    return q_out


# Prefill attention kernel: "flash" = LDS-staged 32x32x16-MFMA flash kernel
# (flash_prefill.hip, tiles of 128 / G tokens); "v1" = the round-1 per-wave kernel
# (attention.hip, tiles of 64 / G ... 8 tokens; kept for A/B runs).
PREFILL_IMPL = os.environ.get("ATTA_PREFILL_IMPL", "flash")
# the flash kernel stages a sequence's whole block-table row in LDS (kBtLds entries: 32k
# tokens at block size 16); wider tables take the v1 kernel
FLASH_MAX_BT = 2048
# waves per flash-prefill workgroup (ops/csrc/flash_prefill.hip NW)
FLASH_WAVES = int(os.environ.get("ATTA_FLASH_WAVES", "4"))
if FLASH_WAVES not in (4, 8):  # the host tiles must match what the kernel covers
    raise ValueError(f"ATTA_FLASH_WAVES={FLASH_WAVES}: flash prefill runs 4 or 8 waves")


def prefill_impl(bt_width: int = 0, impl: str | None = None) -> str:
    """The prefill attention kernel for block tables of ``bt_width`` entries: the configured
    default falls back to v1 past FLASH_MAX_BT; an explicit "flash" there is an error (the
    caller's tiles would not match the kernel that runs)."""
    if impl == "flash" and bt_width > FLASH_MAX_BT:
        raise ValueError(f"flash prefill stages at most {FLASH_MAX_BT} block-table entries "
                         f"per sequence (got {bt_width}); use impl=None or 'v1'")
    impl = impl or PREFILL_IMPL
    return "v1" if impl == "flash" and bt_width > FLASH_MAX_BT else impl


def prefill_tile_tokens(g: int, impl: str | None = None, bt_width: int = 0) -> int:
    """Query tokens per prefill attention workgroup for GQA group ``g``."""
    impl = prefill_impl(bt_width, impl)
    # FLASH_WAVES x (32 // g) tokens (flash: 32 columns per wave) or 4 x (16 // g) (v1: 16) -
    # the G heads of a token share a wave; G = 3 (Llama-3.2-3B) leaves 2 resp. 1 columns idle
    if (impl or PREFILL_IMPL) == "flash":
        return FLASH_WAVES * (32 // g)
    return 4 * (16 // g)


def set_flash_waves(nw: int) -> None:
    """Waves per flash-prefill workgroup (4, or 8: each staged K/V block serves 256 columns).
    Engines build their prefill tiles from prefill_tile_tokens at start: set this before."""
    global FLASH_WAVES
    if nw not in (4, 8):
        raise ValueError("flash prefill runs 4 or 8 waves per workgroup")
    FLASH_WAVES = nw
    if native_available():
        _native().set_flash_waves(nw)


def attention_prefill(q, k_cache, v_cache, block_tables, seq_kvlen, seq_qstart, tile_seq,
                      tile_qoff, scale, out=None, impl: str | None = None,
                      kv_splits: int | None = None):
    """Causal varlen prefill attention over the paged cache.  ``tile_seq`` / ``tile_qoff``
    must come from tiles of ``prefill_tile_tokens(G, impl)`` tokens.  ``kv_splits`` (flash
    only): workgroups per (tile, KV head) over disjoint key ranges; None = ``flash_kv_splits``."""
    check_paged_args(k_cache, block_tables, seq_kvlen, what="attention_prefill")
    if not q.is_cuda:
        return ref.paged_attention(q, k_cache, v_cache, block_tables, seq_kvlen, seq_qstart,
                                   scale, out=out)
    out = torch.empty_like(q) if out is None else out
    if prefill_impl(block_tables.shape[1], impl) != "flash":
        _native().attention_prefill(out, q, k_cache, v_cache, block_tables, seq_kvlen,
                                    seq_qstart, tile_seq, tile_qoff, q.shape[1],
                                    k_cache.shape[1], scale)
        return out
    pairs = tile_seq.shape[0] * k_cache.shape[1]
    ns = flash_kv_splits(pairs) if kv_splits is None else int(kv_splits)
    part = counters = None
    if ns > 1:
        part = torch.empty(pairs * ns * 16640, dtype=torch.float32, device=q.device)
        counters = _flash_counters(q.device, pairs)
    _native().flash_prefill(out, q, k_cache, v_cache, block_tables, seq_kvlen, seq_qstart,
                            tile_seq, tile_qoff, q.shape[1], k_cache.shape[1], scale, ns, part,
                            counters)
    return out


# split-KV flash prefill: steps with few (tile, KV head) pairs over long cached prefixes (a short
# suffix on a multi-thousand-token context leaves most CUs idle while each workgroup walks every
# key block in turn) run up to FLASH_KV_SPLITS workgroups per pair over contiguous key ranges of
# >= 8 blocks (decided per tile on the device) merged by the last arriver.  At the fan-out
# bursts' ~600 keys it measured a wash (5 x 17 rows: 18.2 -> 16.5 us at 32 heads, 19.9 -> 21.2 at
# 64; planning 10.1 -> 11.4 us), so those stay unsplit.  Long prefixes: 17 new rows over 4113
# keys 91.3 -> 34.7 us, 33 over 8209 keys 188.6 -> 65.4 us at 4 splits
# (profiles/r6_flash_split_kv.txt).
# ATTA_FLASH_KV_SPLITS: 0 = auto, 1 = off, n = at most n
FLASH_KV_SPLITS = int(os.environ.get("ATTA_FLASH_KV_SPLITS", "0"))
# fewest 64-key blocks per split (ATTA_FLASH_SPLIT_BLOCKS; a tile splits nblocks // this ways)
FLASH_SPLIT_BLOCKS = int(os.environ.get("ATTA_FLASH_SPLIT_BLOCKS", "8"))
_FLASH_COUNTERS: dict = {}


def flash_kv_splits(pairs: int) -> int:
    if FLASH_KV_SPLITS == 1 or pairs > 128:
        return 1
    cap = FLASH_KV_SPLITS if FLASH_KV_SPLITS > 1 else 8
    return max(1, min(cap, 8, 256 // max(pairs, 1)))


def _flash_counters(device, n: int) -> torch.Tensor:
    """Zeroed arrival counters of the split-KV merge (re-armed by the kernel's last arrivers)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    c = _FLASH_COUNTERS.get(idx)
    if c is None or c.numel() < n:
        c = torch.zeros(max(n, 4096), dtype=torch.int32, device=device)
        _FLASH_COUNTERS[idx] = c
    return c


def attention_decode(q, k_cache, v_cache, block_tables, seq_kvlen, seq_qstart, scale,
                     part_out, part_lse, num_parts, part_tokens, out=None, num_seqs: int = -1):
    """Decode attention for sequences [0, num_seqs) (one query token each)."""
    check_paged_args(k_cache, block_tables, seq_kvlen, num_seqs, "attention_decode")
    if not q.is_cuda:
        n = seq_kvlen.shape[0] if num_seqs < 0 else num_seqs
        return ref.paged_attention(q, k_cache, v_cache, block_tables[:n], seq_kvlen[:n],
                                   seq_qstart[:n + 1], scale, out=out)
    out = torch.empty_like(q) if out is None else out
    _native().attention_decode(out, part_out, part_lse, q, k_cache, v_cache, block_tables,
                               seq_kvlen, seq_qstart, num_seqs, num_parts, part_tokens, q.shape[1],
                               k_cache.shape[1], scale)
    return out


def sample_topkp(logits, temperature, top_p, top_k, seeds, steps, out=None):
    """top-k / top-p sampling, one workgroup per row (ops/csrc/sampling.hip): exact radix-select
    thresholds, the same seeded Gumbel draw as ``sample`` (rows with both filters off get the
    same token), device-side parameters - graph-capturable."""
    if not logits.is_cuda:
        r = ref.sample_topkp(logits, temperature, top_p, top_k, seeds, steps)
        if out is not None:
            out[:r.shape[0]].copy_(r)
            return out[:r.shape[0]]
        return r
    if out is None:
        out = torch.empty(logits.shape[0], dtype=torch.long, device=logits.device)
    _native().sample_topkp(out, logits, temperature, top_p, top_k, seeds, steps)
    return out[:logits.shape[0]]


def sample(logits, temperature, seeds, steps, out=None):
    if not logits.is_cuda:
        r = ref.sample(logits, temperature, seeds, steps)
        if out is not None:
            out.copy_(r)
            return out
        return r
    if out is None:
        out = torch.empty(logits.shape[0], dtype=torch.long, device=logits.device)
    _native().sample(out, logits, temperature, seeds, steps)
    return out



# skinny-GEMM (decode) dispatch: rows <= SKINNY_MAX_M use the MFMA weight-streaming kernel,
# larger M (prefill) goes to hipBLASLt through F.linear.
SKINNY_MAX_M = int(os.environ.get("ATTA_SKINNY_MAX_M", "32"))
# 33..WIDE_MAX_M rows over PRE-SHUFFLED 16-bit weights run the wide small-M kernel
# (csrc/wide.hip: x staged once per workgroup in LDS and shared by its tiles, split-K for the
# narrow projections), with the same fused epilogues - burst prefills and decode batches of
# up to 128 sequences.  0 (or anything <= SKINNY_MAX_M) turns it off.
WIDE_MAX_M = int(os.environ.get("ATTA_WIDE_MAX_M", "128"))
# 129..MIDM_MAX_M rows over pre-shuffled 16-bit weights run the mid-M kernel (csrc/midm.h:
# row-blocked BM x 128 tiles, ~256 workgroups, the same fused epilogues) - the uncached burst
# and planning prefills.  Needs the wide kernel on up to 128 rows; 0 turns it off.
MIDM_MAX_M = int(os.environ.get("ATTA_MIDM_MAX_M", "1024"))


def fused_max_rows(preshuffled: bool = True, fp8: bool = False) -> int:
    """Most rows a call may have to run on the hand-written weight-streaming kernels (the
    16-row-tile GEMVs, the wide small-M kernel, the mid-M kernel) for this weight format:
    pre-shuffled 16-bit or fp8 weights (the W8 builds of the wide / mid-M kernels)."""
    del fp8  # both kernels have fp8-weight builds
    if not preshuffled or WIDE_MAX_M <= SKINNY_MAX_M:
        return SKINNY_MAX_M
    if WIDE_MAX_M >= 128 and MIDM_MAX_M > 128:
        return MIDM_MAX_M
    return min(WIDE_MAX_M, 128)


SKINNY_WAVES = int(os.environ.get("ATTA_SKINNY_WAVES", "8"))
# per-projection wave counts from the MI355X sweep (profiles/r1_microbench_v3_plain.txt):
# 8 waves x 2-deep stages for the small qkv / o projections, 16 waves for the large ones.
WAVES_SMALL = int(os.environ.get("ATTA_WAVES_SMALL", "8"))
WAVES_LARGE = int(os.environ.get("ATTA_WAVES_LARGE", "16"))

# Workgroup waves per decode projection and weight format, from cold-cache sweeps on MI355X
# (profiles/r1_microbench_v5_cold_preshuffle.txt, r1_microbench_v6_fp8.txt, and the
# pre-shuffled unroll sweep): "rm" row-major 16-bit, "ps" pre-shuffled 16-bit, "fp8".
DECODE_WAVES = {
    "qkv": {"rm": 8, "ps": 4, "fp8": 8},
    "o": {"rm": 8, "ps": 8, "fp8": 8},
    "gate_up": {"rm": 16, "ps": 16, "fp8": 8},
    "down": {"rm": 16, "ps": 8, "fp8": 16},
    "lm_head": {"rm": 16, "ps": 16, "fp8": 16},
}
# tuning override: ATTA_DECODE_WAVES="qkv.ps=8,down.fp8=16"
for _item in filter(None, os.environ.get("ATTA_DECODE_WAVES", "").split(",")):
    _key, _, _val = _item.partition("=")
    _proj, _, _fmt = _key.strip().partition(".")
    DECODE_WAVES[_proj][_fmt] = int(_val)


# 17-32 rows (two MFMA row blocks: the fused small-prefill path) stream gate_up best with 8
# waves - half the per-workgroup cross-wave reduction per weight byte: 71.8 -> 59.2 us at 17
# rows, while 16 waves stay best at <= 16 rows (profiles/r4_skinny_mt_probe.txt)
DECODE_WAVES_MT2 = {"gate_up": 8}


def decode_waves(proj: str, preshuffled: bool = False, fp8: bool = False, m: int = 0) -> int:
    if m > 16 and preshuffled and not fp8 and proj in DECODE_WAVES_MT2:
        return DECODE_WAVES_MT2[proj]
    return DECODE_WAVES[proj]["fp8" if fp8 else ("ps" if preshuffled else "rm")]


# Split-K factor per decode projection: gridDim.y slices of K per 16-column tile so grids
# that leave CUs idle (qkv: 384 tiles, o / down: 256 tiles on 256 CUs) stream from every CU;
# the tile's last slice combines the fp32 partials in slice order (ops/csrc/gemv.hip).
# 0 = auto (``auto_ksplit``).  The MI355X sweep (profiles/r2_microbench_splitk.txt) shows the
# in-launch combine costs ~1.5-2 us, so splitting only pays when the grid is far below the
# CU count: Llama-3.1-8B shapes (>= 256 tiles) all run fastest unsplit, the 70B TP=8 qkv
# shard (80 tiles, K 8192) runs 14.7 -> 8.7 us at split 2.
DECODE_KSPLIT = {"qkv": 0, "o": 0, "gate_up": 0, "down": 0}
for _item in filter(None, os.environ.get("ATTA_DECODE_KSPLIT", "").split(",")):
    _key, _, _val = _item.partition("=")
    DECODE_KSPLIT[_key.strip()] = int(_val)


def auto_ksplit(tiles: int, K: int) -> int:
    """Split so a small grid reaches >= ~160 workgroups, keeping >= 2048 of K per slice."""
    ks = 1
    while tiles * ks < 160 and K // (ks * 2) >= 2048:
        ks *= 2
    return ks

# wide-kernel split-K slabs in bf16 (ATTA_SPLITK_HALF=1): half the slab traffic of the
# qkv / o / down launches at 33-128 rows, each slice's partial rounded to bf16 once before the
# fp32 slice-ordered sum
SPLITK_HALF = int(os.environ.get("ATTA_SPLITK_HALF", "0"))


def set_splitk_half(on: bool) -> None:
    """bf16 (True) or fp32 (False) split-K slabs for the wide kernel's following launches."""
    global SPLITK_HALF
    SPLITK_HALF = int(bool(on))
    _native().set_splitk_half(SPLITK_HALF)


SPLITK_WS_FLOATS = 16 << 20  # 64 MiB: tiles x split x rows x 16 fp32 slots (mid-M splits)
SPLITK_COUNTERS = 8192
_SPLITK_WS: dict = {}


def ensure_splitk_workspace(device) -> None:
    """Allocate + register the split-K workspace of ``device`` once (before any capture:
    captured launches keep its address for the life of the graph)."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx in _SPLITK_WS:
        return
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("split-K workspace must be allocated before hipGraph capture")
    ws = torch.zeros(SPLITK_WS_FLOATS, dtype=torch.float32, device=f"cuda:{idx}")
    counters = torch.zeros(SPLITK_COUNTERS, dtype=torch.int32, device=f"cuda:{idx}")
    _native().set_splitk_workspace(ws, counters)
    _SPLITK_WS[idx] = (ws, counters)


def _ksplit(proj: str, x: torch.Tensor, ksplit: int | None, tiles: int) -> int:
    k = DECODE_KSPLIT.get(proj, 0) if ksplit is None else ksplit
    if k <= 0:
        k = auto_ksplit(tiles, x.shape[1])
    if k > 1:
        ensure_splitk_workspace(x.device)
    return k


def skinny_ok(x: torch.Tensor, w: torch.Tensor, preshuffled: bool = False,
              fp8: bool = False) -> bool:
    """Does ``x @ w.T`` run on the hand-written MFMA kernels?  <= SKINNY_MAX_M rows on any
    16-bit / fp8 layout (gemv.hip); up to ``fused_max_rows()`` rows on pre-shuffled 16-bit
    weights (wide.hip to 128 rows, midm.hip beyond)."""
    m, k = x.shape
    lim = fused_max_rows(preshuffled, fp8)
    return (x.is_cuda and 1 <= m <= lim and w.shape[0] % 16 == 0
            and k % 128 == 0 and x.stride(1) == 1 and w.is_contiguous())


def set_wide_plan(waves: int = 0, ksplit: int = 0) -> None:
    """Override the (waves = 16-column tiles per workgroup, K split) plan of the NEXT wide
    small-M launch (tuning sweeps); 0 = the kernel library's own plan."""
    _native().set_wide_plan(int(waves), int(ksplit))


def set_midm_plan(bmt: int = 0, ksplit: int = 0) -> None:
    """Override the (row-block height 16 * bmt, K slices) plan of the NEXT mid-M launch
    (tuning sweeps, warm-up); 0 = the kernel library's own plan."""
    _native().set_midm_plan(int(bmt), int(ksplit))


def midm_plan(m: int, ntiles: int, k: int, epi: int) -> tuple[int, int]:
    """(bmt, K slices) the mid-M kernel plans for m rows x ntiles 16-column tiles x K (epi:
    0 plain, 1 residual add, 2 qkv + RoPE, 3 gate_up + SiLU)."""
    b, s = _native().midm_plan(int(m), int(ntiles), int(k), int(epi), SPLITK_WS_FLOATS)
    return int(b), int(s)


MIDM_BUILT = (3, 4, 5, 6, 8, 10, 12)  # row-block heights / 16 (csrc/midm_b<N>.hip)


def warm_wide_kernels(device, dtype=torch.bfloat16) -> None:
    """Launch one tiny GEMM from every translation unit of the wide (wide_mt<N>.hip: one per
    16-row block count the limits allow) and mid-M kernels (midm_b<N>.hip per row-block
    height, midm.hip's split-K reduce), so every code object is loaded at engine start: HIP
    loads a translation unit's code object at the first launch of one of its kernels, which
    otherwise lands inside a timed prefill (1.5-2.5 ms per object: burst TTFT 4.7 -> 6.3 / 7.3
    ms the first time a 50 / 95-row burst ran, scripts/gpu/probe_fanout_ttft.py).  Only
    kernels the configured limits can route to are launched, and the caller's wide row
    thresholds are restored afterwards."""
    dev = torch.device(device)
    top = fused_max_rows(True, False)
    if dev.type != "cuda" or top <= SKINNY_MAX_M:
        return
    ensure_splitk_workspace(dev)
    w = preshuffle(torch.zeros(128, 256, dtype=dtype, device=dev))
    prev = [int(v) for v in _native().get_wide_min_rows()]
    set_wide_min_rows(1, 1)
    try:
        for mt in range(1, 9):
            if 16 * mt <= min(top, 128):
                linear(torch.zeros(16 * mt, 256, dtype=dtype, device=dev), w, preshuffled=True)
        if top > 128:
            x = torch.zeros(144, 256, dtype=dtype, device=dev)
            for b in MIDM_BUILT:
                set_midm_plan(b, 1)
                linear(x, w, preshuffled=True)
            set_midm_plan(6, 2)  # the split-K reduce launch (midm.hip)
            linear(x, w, preshuffled=True)
    finally:
        set_wide_min_rows(*prev)
    torch.cuda.synchronize(dev)


def set_wide_min_rows(m: int = 17, m_silu: int = 12) -> None:
    """Pre-shuffled 16-bit GEMV calls of >= ``m`` rows (gate_up + SiLU: ``m_silu``) run the
    wide small-M kernel; calls over 32 rows always do.  Defaults = the measured crossover
    (profiles/r5_wide_vs_skinny.txt); 33 / 33 keeps <= 32 rows on the 16-row-tile GEMVs."""
    _native().set_wide_min_rows(int(m), int(m_silu))


def preshuffle(w: torch.Tensor, rowmap: str = "plain") -> torch.Tensor:
    """Re-lay a [N, K] weight for the decode GEMV: rows permuted into the kernel's tile order
    (``rowmap`` "plain" | "qkv" (RoPE pairs d, d+64 of each 128-dim head in one tile) |
    "silu" (gate_j and up_j in one tile)), then every 16-row x 32-column block stored as the
    1 KiB the 64 MFMA lanes load (lane l: row l & 15, columns 8*(l >> 4)..+7).  Same shape
    and dtype as ``w``; only valid as the ``w`` of ops called with ``preshuffled=True``."""
    N, K = w.shape
    if N % 16 or K % 32:
        raise ValueError(f"preshuffle needs N % 16 == 0 and K % 32 == 0, got {tuple(w.shape)}")
    rows = _rowmap_index(N, rowmap, w.device)
    if rows is not None:
        w = w.index_select(0, rows)
    return (w.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous()
            .reshape(N, K))


# ---- fp8 weight-only quantisation (OCP e4m3fn, per output row) ----------------------------
FP8_MAX = 448.0


def quantize_fp8(w: torch.Tensor, row_amax: torch.Tensor | None = None
                 ) -> tuple[torch.Tensor, torch.Tensor]:
    """[N, K] 16-bit weight -> (uint8 e4m3fn bytes [N, K], fp32 per-row scale [N]).

    ``row_amax`` overrides the per-row |max| the scale is derived from: a TP row-parallel
    shard (o / down, a K slice of every row) passes the FULL row's amax, so every rank
    quantises with the TP=1 scale and TP=N fp8 weights are bit-identical to TP=1's."""
    wf = w.float()
    amax = wf.abs().amax(dim=1) if row_amax is None else row_amax.float().to(wf.device)
    scale = (amax / FP8_MAX).clamp_min(1e-12)
    q = (wf / scale[:, None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
    return q.view(torch.uint8), scale.contiguous()


def dequantize_fp8(q: torch.Tensor, scale: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    return (q.view(torch.float8_e4m3fn).float() * scale[:, None].float()).to(dtype)


def preshuffle_fp8(q: torch.Tensor, rowmap: str = "plain") -> torch.Tensor:
    """fp8 analogue of ``preshuffle``: rows permuted by ``rowmap``, then each 16-row x 64-col
    block stored as 64 lanes x 16 bytes, lane l = (row l & 15) holding its 8 k-values of the
    two 32-wide K steps (k = 8*(l >> 4) + j and 32 + 8*(l >> 4) + j)."""
    N, K = q.shape
    if N % 16 or K % 64:
        raise ValueError(f"fp8 preshuffle needs N % 16 == 0 and K % 64 == 0, got {tuple(q.shape)}")
    rows = _rowmap_index(N, rowmap, q.device)
    if rows is not None:
        q = q.index_select(0, rows)
    return (q.reshape(N // 16, 16, K // 64, 2, 4, 8).permute(0, 2, 4, 1, 3, 5).contiguous()
            .reshape(N, K))


def _rowmap_index(N: int, rowmap: str, dev):
    if rowmap == "plain":
        return None
    if rowmap == "qkv":
        if N % 128:
            raise ValueError("qkv rowmap needs whole 128-dim heads")
        t = torch.arange(N // 16, device=dev)
        c = torch.arange(16, device=dev)
        head, j = (t >> 3)[:, None], (t & 7)[:, None]
        return (head * 128 + j * 8 + (c & 7)[None, :] + ((c & 8) != 0)[None, :] * 64).reshape(-1)
    if rowmap == "silu":
        inter = N // 2
        if inter % 8:
            raise ValueError("silu rowmap needs inter % 8 == 0")
        t = torch.arange(inter // 8, device=dev)[:, None]
        c = torch.arange(16, device=dev)[None, :]
        return torch.where(c < 8, t * 8 + c, inter + t * 8 + c - 8).reshape(-1)
    raise ValueError(f"unknown rowmap {rowmap}")


# fp8 activation quantisation modes (ops/csrc/quant_fp8.hip)
QUANT_NORM, QUANT_SILU, QUANT_PLAIN, QUANT_ADDNORM = 0, 1, 2, 3


def quant_rows_fp8(x: torch.Tensor, mode: int = QUANT_PLAIN, w: torch.Tensor | None = None,
                   eps: float = 1e-5, residual: torch.Tensor | None = None
                   ) -> tuple[torch.Tensor, torch.Tensor]:
    """Row-wise e4m3fn quantisation of ``x`` (``QUANT_PLAIN``), of rmsnorm(x) * w
    (``QUANT_NORM``), of silu(gate) * up for gate | up rows (``QUANT_SILU``), or - with
    ``QUANT_ADDNORM`` - ``residual += x`` (in place) then rmsnorm(residual) * w, fused in one
    HIP kernel.  Returns (uint8 codes [M, width], fp32 scales [M, 1])."""
    M = x.shape[0]
    width = x.shape[1] // 2 if mode == QUANT_SILU else x.shape[1]
    if not x.is_cuda:
        if mode == QUANT_ADDNORM:
            residual.copy_((x.float() + residual.float()).to(residual.dtype))
            x, mode = residual, QUANT_NORM
        if mode == QUANT_NORM:
            v = ref.rms_norm(x, w, eps).float()
        elif mode == QUANT_SILU:
            v = ref.silu_and_mul(x).float()
        else:
            v = x.float()
        s = (v.abs().amax(dim=1, keepdim=True) / FP8_MAX)
        s = torch.where(s > 0, s, torch.ones_like(s))
        q = (v / s).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).view(torch.uint8)
        return q, s
    q = torch.empty(M, width, dtype=torch.uint8, device=x.device)
    s = torch.empty(M, 1, dtype=torch.float32, device=x.device)
    _native().quant_rows_fp8(q, s, x, w if mode in (QUANT_NORM, QUANT_ADDNORM) else None, mode,
                             eps, residual if mode == QUANT_ADDNORM else None)
    return q, s


def gemm_fp8(xq: torch.Tensor, xs: torch.Tensor, wq: torch.Tensor, ws: torch.Tensor,
             out_dtype=torch.bfloat16) -> torch.Tensor:
    """y[m, n] = xs[m] ws[n] sum_k fp8(xq)[m, k] fp8(wq)[n, k]: one hipBLASLt fp8 GEMM with
    row-wise scales on both operands (torch._scaled_mm, CDNA4 fp8 MFMA), bf16 out, no torch
    passes around it.  Failures raise: there is no silent dequantise fallback on a GPU."""
    if not xq.is_cuda:
        x = xq.view(torch.float8_e4m3fn).float() * xs
        w = wq.view(torch.float8_e4m3fn).float() * ws.reshape(-1, 1)
        return (x @ w.t()).to(out_dtype)
    return torch._scaled_mm(xq.view(torch.float8_e4m3fn), wq.view(torch.float8_e4m3fn).t(),
                            scale_a=xs, scale_b=ws.reshape(1, -1), out_dtype=out_dtype)


def linear_fp8(x: torch.Tensor, q: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    """y = x @ dequant(q).T for 16-bit activations and row-major fp8 weights: the fused
    row-wise activation quantiser, then ``gemm_fp8``."""
    xq, xs = quant_rows_fp8(x, QUANT_PLAIN)
    return gemm_fp8(xq, xs, q, scale, x.dtype)


GEMM_PLAIN, GEMM_RESADD, GEMM_SILU = 0, 1, 2


def prefill_gemm_ok(x: torch.Tensor, w: torch.Tensor, mode: int = GEMM_PLAIN) -> bool:
    """Shapes the hand-written prefill GEMM (ops/csrc/prefill_gemm.hip) takes: bf16 or fp8
    (uint8 e4m3fn) operands, K a multiple of 64 bytes, output width a multiple of 256 (128
    for the SiLU mode), 16-B aligned rows."""
    n = w.shape[0] // 2 if mode == GEMM_SILU else w.shape[0]
    el = x.element_size()
    return (x.dtype in (torch.bfloat16, torch.uint8) and w.dtype == x.dtype and x.dim() == 2
            and x.shape[1] == w.shape[1] and (x.shape[1] * el) % 64 == 0 and x.stride(1) == 1
            and (x.stride(0) * el) % 16 == 0 and w.is_contiguous()
            and n % (128 if mode == GEMM_SILU else 256) == 0)


_PG_SCHEDULES = {"hybrid": 0, "streamk": 1, "dp": 2, "splitk": 3}


def prefill_gemm(x: torch.Tensor, w: torch.Tensor, mode: int = GEMM_PLAIN,
                 residual: torch.Tensor | None = None, out: torch.Tensor | None = None,
                 xs: torch.Tensor | None = None, ws: torch.Tensor | None = None,
                 schedule: str | None = None, bm: int = 0) -> torch.Tensor:
    """Hand-written CDNA4 prefill GEMM: ``x @ w.T`` (GEMM_PLAIN), ``residual += x @ w.T`` in
    place (GEMM_RESADD; returns ``residual``) or ``silu(x @ gate.T) * (x @ up.T)`` for
    ``w = [gate; up]`` (GEMM_SILU).  bf16 operands, or fp8: uint8 e4m3fn ``x`` / ``w`` with
    fp32 row scales ``xs`` [M, 1] / ``ws`` [rows of w] (applied in the epilogue).  fp32
    accumulate, one rounding to bf16.  ``schedule`` (hybrid / streamk / dp / splitk) and ``bm``
    (tile height 64 / 128 / 256; 0 = by row count) apply to this call only - nothing
    process-wide changes.  CPU tensors run the PyTorch reference of the op."""
    n = w.shape[0] // 2 if mode == GEMM_SILU else w.shape[0]
    fp8 = x.dtype == torch.uint8
    if fp8 and (xs is None or ws is None):
        raise ValueError("prefill_gemm: fp8 operands need row scales xs and ws")
    if not x.is_cuda:
        if fp8:
            xf = x.view(torch.float8_e4m3fn).float() * xs.reshape(-1, 1)
            wf = w.view(torch.float8_e4m3fn).float() * ws.reshape(-1, 1)
        else:
            xf, wf = x.float(), w.float()
        y = xf @ wf.t()
        if mode == GEMM_SILU:
            y = torch.nn.functional.silu(y[:, :n]) * y[:, n:]
        if mode == GEMM_RESADD:
            residual.copy_((y + residual.float()).to(residual.dtype))
            return residual
        y = y.to(torch.bfloat16)
        if out is not None:
            out.copy_(y)
            return out
        return y
    sched = -1 if schedule is None else _PG_SCHEDULES[schedule]
    xs_ = xs.reshape(-1) if fp8 else None
    ws_ = ws.reshape(-1) if fp8 else None
    if mode == GEMM_RESADD:
        _native().prefill_gemm(residual, x, w, residual, mode, xs_, ws_, sched, bm)
        return residual
    if out is None:
        out = torch.empty(x.shape[0], n, dtype=torch.bfloat16, device=x.device)
    _native().prefill_gemm(out, x, w, None, mode, xs_, ws_, sched, bm)
    return out


_PG_SCHEDULE = "hybrid"  # the configured (process-wide) default schedule


def prefill_gemm_config(schedule: str = "hybrid", group_m: int = 4, ablate: int = 0) -> None:
    """Process-wide defaults of the prefill GEMM: schedule "hybrid" (data-parallel rounds +
    Stream-K remainder), "streamk", "dp" or "splitk" (co-resident K slices of a few whole
    tiles with a parallel reduction, where T * S fits the CUs); ``group_m`` M tiles per raster
    group; ``ablate`` (measurement only, bf16 plain GEMMs): 1 no MFMA, 2 no LDS-DMA, 3 no
    ds_read; 4 (tests): every cross-workgroup wait gives up at once (recompute fallback)."""
    global _PG_SCHEDULE
    _native().prefill_gemm_config(_PG_SCHEDULES[schedule], group_m, ablate)
    _PG_SCHEDULE = schedule


def prefill_gemm_auto_bm(m: int) -> int:
    """Tile height the library picks for m rows (fewest padding rows)."""
    return int(_native().prefill_gemm_auto_bm(m))


def prefill_gemm_error() -> int:
    """Nonzero once a cross-workgroup wait of the prefill GEMM timed out (bit 1 stream-K,
    bit 2 split-K); bit 4 says the waiting workgroup recomputed its tile itself, so the
    outputs are still exact."""
    return int(_native().prefill_gemm_error())


def prefill_gemm_error_to(host: torch.Tensor, clear: bool = True) -> None:
    """Enqueue a copy of the prefill GEMM's error word into ``host`` (pinned int32) on the
    current stream; read it after the next synchronisation (no extra sync of its own).
    ``clear``: zero the word behind the copy, so each read covers the calls since the last."""
    _native().prefill_gemm_error_to(host, bool(clear))


def prefill_gemm_error_reset() -> None:
    """Zero the prefill GEMM's error word."""
    _native().prefill_gemm_error_reset()


def _need_cuda(x, preshuffled):
    if preshuffled and not x.is_cuda:
        raise ValueError("pre-shuffled weights are only consumed by the HIP decode kernels")


def linear(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor | None = None,
           out: torch.Tensor | None = None, waves: int | None = None,
           preshuffled: bool = False, w_scale: torch.Tensor | None = None,
           ksplit: int | None = 1, proj: str = "") -> torch.Tensor:
    """y = x @ w.T.  With ``residual`` the product is added to ``residual`` IN PLACE and
    ``residual`` is returned (residual-stream update).  Decode-sized M runs the MFMA skinny
    GEMM; everything else (prefill, CPU) runs F.linear (hipBLASLt on the GPU).
    ``preshuffled``: ``w`` comes from ``preshuffle`` (skinny path only).
    ``w_scale``: ``w`` is fp8 (uint8, ``preshuffle_fp8`` layout) with this per-row scale."""
    _need_cuda(x, preshuffled or w_scale is not None)
    fp8 = w_scale is not None
    if fp8:
        preshuffled = True
    if preshuffled and not skinny_ok(x, w, preshuffled, fp8):
        raise ValueError("pre-shuffled weights need the skinny (decode) path")
    if skinny_ok(x, w, preshuffled, fp8):
        ksplit = _ksplit(proj, x, ksplit, w.shape[0] // 16)
        if residual is not None:
            _native().skinny_gemm(residual, x, w, residual, waves or SKINNY_WAVES, preshuffled,
                                  w_scale, ksplit)
            return residual
        if out is None:
            out = torch.empty(x.shape[0], w.shape[0], dtype=x.dtype, device=x.device)
        _native().skinny_gemm(out, x, w, None, waves or SKINNY_WAVES, preshuffled, w_scale,
                              ksplit)
        return out
    if residual is not None:
        # hipBLASLt C-matrix epilogue: residual = residual + x @ w.T in one GEMM (fp32
        # accumulate, one rounding), no separate add pass over the residual stream
        if residual.is_cuda:
            return residual.addmm_(x, w.t())
        residual.copy_((torch.nn.functional.linear(x, w).float() + residual.float())
                       .to(residual.dtype))
        return residual
    y = torch.nn.functional.linear(x, w)
    if out is not None:
        out.copy_(y)
        return out
    return y


def linear_push_reduce(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor, ipc,
                       waves: int | None = None, preshuffled: bool = False,
                       w_scale: torch.Tensor | None = None, proj: str = "") -> torch.Tensor:
    """TP row-parallel projection with the all-reduce push fused into the decode GEMV
    (SURVEY §2.5 X1 / X2): the GEMV epilogue writes this rank's partial product into every
    rank's IPC receive slot, then one receive kernel adds the rank-order sum into
    ``residual`` (returned).  ``ipc``: the TP group's IpcAllReduce."""
    if w_scale is not None:
        preshuffled = True
    if not skinny_ok(x, w):
        raise ValueError("linear_push_reduce: decode-sized rows only")
    n_out = w.shape[0]
    ksplit = _ksplit(proj, x, None, n_out // 16)
    ipc.gemv_push(x, w, n_out, waves or SKINNY_WAVES, preshuffled, w_scale, ksplit)
    return ipc.push_reduce(residual, n_out)


# ---- fused decode-step ops (norm weight folded into W on the host) -----------------------
def decode_qkv_rope(x, w, eps, positions, slots, cos_sin, k_cache, v_cache, n_q_heads,
                    n_kv_heads, q_out=None, preshuffled=False, w_scale=None, ksplit=None):
    """RMSNorm(x) -> QKV GEMM -> RoPE -> q out + paged K/V write, one kernel on the GPU."""
    _need_cuda(x, preshuffled or w_scale is not None)
    check_slots(k_cache, slots[:x.shape[0]], "decode_qkv_rope")
    if q_out is None:
        q_out = torch.empty(x.shape[0], n_q_heads, 128, dtype=x.dtype, device=x.device)
    if not x.is_cuda:
        n = ref.rms_norm(x, torch.ones(x.shape[1], dtype=x.dtype), eps)
        q = ref.rope_cache(torch.nn.functional.linear(n, w), positions, slots, cos_sin, k_cache,
                           v_cache, n_q_heads, n_kv_heads, 128)
        q_out.copy_(q)
        return q_out
    _native().fused_qkv_rope(q_out, k_cache, v_cache, x, w, positions, slots, cos_sin,
                             n_q_heads, n_kv_heads, eps,
                             decode_waves("qkv", preshuffled, w_scale is not None),
                             preshuffled or w_scale is not None, w_scale,
                             _ksplit("qkv", x, ksplit, w.shape[0] // 16))
    return q_out


def decode_gate_up_silu(x, w, eps, out=None, preshuffled=False, w_scale=None, ksplit=None):
    """RMSNorm(x) -> gate_up GEMM -> SiLU(gate) * up, one kernel on the GPU."""
    _need_cuda(x, preshuffled or w_scale is not None)
    inter = w.shape[0] // 2
    if out is None:
        out = torch.empty(x.shape[0], inter, dtype=x.dtype, device=x.device)
    if not x.is_cuda:
        n = ref.rms_norm(x, torch.ones(x.shape[1], dtype=x.dtype), eps)
        out.copy_(ref.silu_and_mul(torch.nn.functional.linear(n, w)))
        return out
    waves = decode_waves("gate_up", preshuffled, w_scale is not None, m=x.shape[0])
    _native().fused_gate_up_silu(out, x, w, eps, waves, preshuffled or w_scale is not None,
                                 w_scale, _ksplit("gate_up", x, ksplit, w.shape[0] // 16))
    return out


def decode_lm_head_sample(x, w, eps, temperature, seeds, steps, keys, tokens=None,
                          finalize=True, vocab_offset=0, preshuffled=False):
    """Final RMSNorm -> LM head -> greedy / Gumbel-max sample without materialising logits.
    ``keys`` (int64, >= M * vocab/16 entries) is scratch for the per-tile packed
    (value, index) maxima; no initialisation is needed.

    ``finalize``: True -> ``tokens`` gets token ids; ``"key"`` -> ``tokens`` gets each row's
    signed-orderable packed key (TP: MAX all-reduce them, then ``key_to_token``); False ->
    partials only.  ``vocab_offset`` is this shard's first vocab id."""
    _need_cuda(x, preshuffled)
    if tokens is None:
        tokens = torch.empty(x.shape[0], dtype=torch.long, device=x.device)
    if not x.is_cuda:
        n = ref.rms_norm(x, torch.ones(x.shape[1], dtype=x.dtype), eps)
        logits = torch.nn.functional.linear(n, w)
        if finalize == "key":
            tokens.copy_(ref.sample_keys(logits, temperature, seeds, steps, vocab_offset))
        else:
            tokens.copy_(ref.sample(logits, temperature, seeds, steps, vocab_offset))
        return tokens
    mode = 2 if finalize == "key" else (1 if finalize else 0)
    _native().fused_lm_head_sample(tokens, keys, x, w, eps, temperature, seeds, steps, mode,
                                   vocab_offset, decode_waves("lm_head", preshuffled),
                                   preshuffled)
    return tokens


def key_to_token(keys: torch.Tensor) -> torch.Tensor:
    """Decode signed-orderable packed sampler keys (``finalize="key"``) to token ids."""
    return 0xFFFFFFFF - (keys & 0xFFFFFFFF)


def set_attention_trace(trace=None):
    """Per-workgroup timeline of the decode attention launches that follow (int64 CUDA tensor
    of 4 words per workgroup of the (seqs, kv heads, partitions) grid: past round trip 1,
    computed, published, end - 100 MHz wall clock); None switches it off."""
    _native().set_attention_trace(trace)


def set_gemv_trace(trace=None):
    """Per-workgroup [start, end] timeline (100 MHz wall clock, int64 CUDA tensor of 2 words
    per workgroup) of the NEXT decode GEMV launch only; None clears it."""
    _native().set_gemv_trace(trace)


def attention_decode_v2(q, k_cache, v_cache, block_tables, seq_kvlen, seq_qstart, scale,
                        part_out, part_lse, counters, max_parts, part_tokens, out=None,
                        num_seqs: int = -1):
    """Decode attention with in-kernel split-K combine (one launch)."""
    check_paged_args(k_cache, block_tables, seq_kvlen, num_seqs, "attention_decode_v2")
    if not q.is_cuda:
        n = seq_kvlen.shape[0] if num_seqs < 0 else num_seqs
        return ref.paged_attention(q, k_cache, v_cache, block_tables[:n], seq_kvlen[:n],
                                   seq_qstart[:n + 1], scale, out=out)
    out = torch.empty_like(q) if out is None else out
    _native().attention_decode_v2(out, part_out, part_lse, counters, q, k_cache, v_cache,
                                  block_tables, seq_kvlen, seq_qstart, num_seqs, max_parts,
                                  part_tokens, q.shape[1], k_cache.shape[1], scale)
    return out
