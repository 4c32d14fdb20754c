"""CPU check of the decode-GEMV weight layout (ops.preshuffle) against its definition."""
import pytest
import torch

from agentic_traffic_testing_amd import ops


def _row(mode, t, c, N):
    if mode == "qkv":
        return (t >> 3) * 128 + (t & 7) * 8 + (c & 7) + (64 if c & 8 else 0)
    if mode == "silu":
        inter = N // 2
        return t * 8 + c if c < 8 else inter + t * 8 + c - 8
    return t * 16 + c


@pytest.mark.parametrize("mode,N,K", [("plain", 64, 96), ("qkv", 256, 64), ("silu", 64, 32)])
def test_preshuffle_layout(mode, N, K):
    w = torch.arange(N * K, dtype=torch.int32).reshape(N, K)
    ps = ops.preshuffle(w, mode).reshape(-1)
    for t in range(N // 16):
        for s in range(K // 32):
            for lane in range(64):
                for j in range(0, 8, 3):
                    got = int(ps[((t * (K // 32) + s) * 512) + lane * 8 + j])
                    exp = int(w[_row(mode, t, lane & 15, N), s * 32 + 8 * (lane >> 4) + j])
                    assert got == exp
    # a permutation of the original elements
    assert torch.equal(torch.sort(ps).values, torch.arange(N * K, dtype=torch.int32))


def test_preshuffle_rejects_bad_shapes_and_cpu_use():
    with pytest.raises(ValueError):
        ops.preshuffle(torch.zeros(10, 32))
    with pytest.raises(ValueError):
        ops.linear(torch.zeros(1, 32), torch.zeros(16, 32), preshuffled=True)


def test_fp8_quantize_roundtrip_and_layout():
    torch.manual_seed(0)
    w = torch.randn(64, 128) * 0.05
    w[3] *= 40  # rows with very different ranges keep their own scale
    q, s = ops.quantize_fp8(w)
    assert q.dtype == torch.uint8 and s.shape == (64,)
    back = ops.dequantize_fp8(q, s, torch.float32)
    rel = ((back - w).abs() / w.abs().amax(dim=1, keepdim=True)).max()
    assert float(rel) < 1 / 16  # e4m3: 3 mantissa bits
    # fp8 pre-shuffle layout against its definition
    N, K = 32, 128
    b = torch.arange(N * K, dtype=torch.int32).reshape(N, K)
    ps = ops.preshuffle_fp8(b, "plain").reshape(-1)
    for t in range(N // 16):
        for kp in range(K // 64):
            for lane in range(64):
                for half in range(2):
                    for j in (0, 7):
                        got = int(ps[(t * (K // 64) + kp) * 1024 + lane * 16 + half * 8 + j])
                        exp = int(b[t * 16 + (lane & 15), kp * 64 + half * 32 + 8 * (lane >> 4) + j])
                        assert got == exp


def test_fp8_engine_cpu_reference():
    """fp8 quantisation on the CPU reference path stores the dequantised values; the engine
    runs end to end and stays close to the 16-bit model's greedy output."""
    from agentic_traffic_testing_amd.config import EngineConfig
    from agentic_traffic_testing_amd.engine.llm_engine import LLMEngine
    from agentic_traffic_testing_amd.engine.sequence import SamplingParams

    base = dict(model="tiny", device="cpu", max_model_len=128, num_kv_blocks=32,
                max_num_batched_tokens=128, max_num_seqs=2, use_graphs=False)
    sp = SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True)
    e8 = LLMEngine(EngineConfig(quantization="fp8", **base))
    e16 = LLMEngine(EngineConfig(**base))
    L8, L16 = e8.runner.model.layers[0], e16.runner.model.layers[0]
    assert L8.qkv.dtype == torch.bfloat16 and not torch.equal(L8.qkv, L16.qkv)
    rel = (L8.qkv.float() - L16.qkv.float()).abs().max() / L16.qkv.float().abs().max()
    assert float(rel) < 0.07
    out = e8.generate([[5, 6, 7, 8, 9, 10]], sp)
    assert len(out[0].token_ids) == 4
