"""Prefill row padding to the tuned-GEMM buckets (agentic_traffic_testing_amd/tuning): the
bucket function, and an engine whose prefill steps are padded produces exactly the tokens of
the unpadded engine (padding rows carry slot -1: never written to the KV cache, never
sampled)."""
import numpy as np

from agentic_traffic_testing_amd import tuning
from agentic_traffic_testing_amd.config import EngineConfig
from agentic_traffic_testing_amd.engine.llm_engine import LLMEngine
from agentic_traffic_testing_amd.engine.sequence import SamplingParams


def test_bucket_rows():
    prev = 0
    for t in range(1, 9000):
        b = tuning.bucket_rows(t)
        assert b >= t and b >= prev
        assert (b - t) <= max(15, t // 4), (t, b)
        if t >= 256:
            assert (b - t) * 8 <= t, (t, b)
        prev = b
    assert tuning.bucket_rows(73) == 80 and tuning.bucket_rows(382) == 384
    assert tuning.bucket_rows(3092) == 3200
    bs = tuning.all_buckets(8192)
    assert bs == sorted(set(bs)) and bs[-1] == 8192
    assert all(tuning.bucket_rows(b) == b for b in bs)


def test_no_table_for_unknown_spec(tmp_path):
    assert tuning.load("", "llama-3.1-8b") is None
    assert tuning.load(str(tmp_path / "missing.csv"), "llama-3.1-8b") is None


def _gen(pad: bool):
    eng = LLMEngine(EngineConfig(model="tiny", device="cpu", max_model_len=256, num_kv_blocks=64,
                                 max_num_batched_tokens=256, max_num_seqs=8, use_graphs=False,
                                 gemm_tuning=""))
    if pad:
        eng.runner.gemm_table = "forced-for-test"  # pad prefill steps as with a loaded table
    rng = np.random.default_rng(3)
    prompts = [rng.integers(300, 3000, size=n).tolist() for n in (37, 5, 70)]
    outs = eng.generate(prompts, SamplingParams(temperature=0.0, max_tokens=5, ignore_eos=True))
    return [o.token_ids for o in outs]


def test_padded_prefill_matches_unpadded():
    assert _gen(True) == _gen(False)


def test_prefill_impl_falls_back_past_flash_table_width():
    """The flash prefill kernel stages a sequence's whole block-table row in LDS: wider tables
    take v1 by default (tile size and kernel chosen together), an explicit flash request fails."""
    import pytest

    from agentic_traffic_testing_amd import ops

    assert ops.prefill_impl(ops.FLASH_MAX_BT, None) == ops.PREFILL_IMPL
    if ops.PREFILL_IMPL == "flash":
        assert ops.prefill_impl(ops.FLASH_MAX_BT + 1, None) == "v1"
        assert ops.prefill_tile_tokens(4, bt_width=ops.FLASH_MAX_BT + 1) == \
            ops.prefill_tile_tokens(4, "v1")
    with pytest.raises(ValueError):
        ops.prefill_impl(ops.FLASH_MAX_BT + 1, "flash")


def _table_shapes(path):
    """{(op kind, m, n, k)} of a TunableOp CSV (tn_<n>_<m>_<k>_...)."""
    out = set()
    for line in open(path):
        p = line.rstrip("\n").split(",")
        if p[0] == "Validator" or len(p) < 4:
            continue
        n, m, k = (int(v) for v in p[1].split("_")[1:4])
        out.add(("fp8" if p[0].startswith("Scaled") else "bf16", m, n, k))
    return out


def test_shipped_tables_cover_every_bucket_and_shard():
    """the shipped tables hold every projection's GEMM at every row bucket up
    to 4096 - the 8B (bf16 and fp8) and the 70B at TP=1 and its TP=8 per-rank shard shapes
    (column-parallel qkv / gate_up split N, row-parallel o / down split K), bf16 and fp8."""
    from agentic_traffic_testing_amd.config import resolve_model
    buckets = tuning.all_buckets(4096)
    for model, tps in (("llama-3.1-8b", (1,)), ("llama-3-70b", (1, 8)),
                       ("llama-3.1-70b", (1, 8))):
        mc = resolve_model(model)[0]
        have = _table_shapes(tuning.table_path(mc.name))
        H, I = mc.hidden_size, mc.intermediate_size
        qkv = (mc.num_heads + 2 * mc.num_kv_heads) * mc.head_dim
        o_k = mc.num_heads * mc.head_dim
        for tp in tps:
            shapes = [(qkv // tp, H), (H, o_k // tp), (2 * I // tp, H), (H, I // tp)]
            for kind in ("bf16", "fp8"):
                miss = [(m, n, k) for m in buckets for n, k in shapes
                        if (kind, m, n, k) not in have]
                assert not miss, (model, tp, kind, miss[:4])
