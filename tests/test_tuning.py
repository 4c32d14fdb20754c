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
