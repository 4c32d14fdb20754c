import torch, sys
sys.path.insert(0, ".")
from agentic_traffic_testing_amd import ops
from agentic_traffic_testing_amd.ops import reference as ref
ops.native_available(); ops.ensure_splitk_workspace("cuda")
torch.manual_seed(53)
dt = torch.bfloat16
for m in (129, 200, 382, 475):
    for plan in ((0, 0), (3, 1), (4, 1), (6, 1), (8, 1)):
        inter, k = 14336, 4096
        torch.manual_seed(53)
        x = torch.randn(m, k, dtype=dt, device="cuda")
        w = torch.randn(2 * inter, k, dtype=dt, device="cuda") * 0.02
        n = ref.rms_norm(x, torch.ones(k, dtype=dt, device="cuda"), 1e-5)
        exp = ref.silu_and_mul(torch.nn.functional.linear(n, w)).float()
        # fp32 oracle on the same normed-x (no bf16 rounding of the GEMM output)
        g = n.float() @ w.float().t()
        o32 = torch.nn.functional.silu(g[:, :inter]) * g[:, inter:]
        ops.set_midm_plan(*plan)
        got = ops.decode_gate_up_silu(x, ops.preshuffle(w, "silu"), 1e-5, preshuffled=True).float()
        err = (got - exp).abs()
        tol = 0.04 + 0.04 * exp.abs()
        bad = (err > tol)
        e32 = (got - o32).abs().max().item()
        eref = (exp - o32).abs().max().item()
        print(m, plan, ops.midm_plan(m, inter // 8, k, 3), "maxerr", err.max().item(), "bad", int(bad.sum()),
              "rows", sorted(set(bad.nonzero()[:, 0].tolist()))[:10], "vs fp32: got", e32, "ref", eref, flush=True)
