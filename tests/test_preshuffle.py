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
