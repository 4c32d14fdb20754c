"""Config-1 CPU backend in --hf-compat mode (serving/hf_compat.py): facebook/opt-125m served as
an OPT model (not a Llama preset) with the reference hf_cpu_server contract
(/root/reference/llm/hf_cpu_server.py:34-51, 86-94): ``{"output": prompt + completion}``,
temperature 0.7 sampling by default.  Parity is pinned against transformers'
OPTForCausalLM built from the same seed - the weights are random-init because there is no
network, so no published checkpoint output covers this ("parity unpinned" beyond it)."""
import asyncio

import pytest
import torch

from agentic_traffic_testing_amd.serving import hf_compat
from agentic_traffic_testing_amd.serving.hf_compat import HFCausalLM, create_app, is_hf_family


@pytest.fixture(scope="module")
def lm():
    return HFCausalLM("facebook/opt-125m", seed=7)


def test_opt125m_architecture(lm):
    from transformers import OPTConfig

    c = lm.config
    assert c.model_type == "opt"
    ref = OPTConfig()
    assert (c.hidden_size, c.num_hidden_layers, c.ffn_dim, c.vocab_size) == (
        ref.hidden_size, ref.num_hidden_layers, ref.ffn_dim, ref.vocab_size) == (768, 12, 3072,
                                                                                 50272)
    assert type(lm.model).__name__ == "OPTForCausalLM"
    n = sum(p.numel() for p in lm.model.parameters())
    assert 120e6 < n < 130e6  # OPT-125m


def test_greedy_parity_with_transformers(lm):
    from transformers import OPTConfig, OPTForCausalLM

    torch.manual_seed(7)
    ref = OPTForCausalLM(OPTConfig()).eval()
    for (k, a), b in zip(lm.model.state_dict().items(), ref.state_dict().values()):
        assert torch.equal(a, b), k
    ids = lm.encode("The agents discussed the plan and")
    got = lm.generate_ids(ids, 8, temperature=0.0, do_sample=False)
    inp = torch.tensor([ids])
    with torch.inference_mode():
        exp = ref.generate(inp, attention_mask=torch.ones_like(inp), max_new_tokens=8,
                           do_sample=False, pad_token_id=lm.eos, eos_token_id=lm.eos)
    assert got == exp[0, len(ids):].tolist()
    # and the logits of one step, directly
    with torch.inference_mode():
        la = lm.model(inp).logits[0, -1]
        lb = ref(inp).logits[0, -1]
    assert torch.allclose(la, lb)
    assert int(la.argmax()) == got[0]


def test_reference_sampling_and_echo(lm):
    text, n_in, n_out = lm.generate("hello agents", 6, seed=3)
    assert text.startswith("hello agents")
    assert 1 <= n_out <= 6 and n_in >= 2
    again, _, _ = lm.generate("hello agents", 6, seed=3)
    assert again == text  # seeded temperature-0.7 draw is reproducible


def test_family_selection():
    assert is_hf_family("facebook/opt-125m") and is_hf_family("gpt2")
    assert not is_hf_family("meta-llama/Llama-3.1-8B-Instruct")
    assert hf_compat.hf_config_for("facebook/opt-350m").hidden_size == 1024


def test_http_contract(lm):
    from aiohttp.test_utils import TestClient, TestServer

    async def go():
        async with TestClient(TestServer(create_app(lm, default_max_tokens=4))) as c:
            r = await c.post("/chat", json={"prompt": "plan the trip", "max_tokens": 3})
            assert r.status == 200
            body = await r.json()
            assert set(body) == {"output"} and body["output"].startswith("plan the trip")
            r = await c.post("/generate", json={"input": "x", "temperature": 0})
            assert r.status == 200
            r = await c.post("/completion", json={"max_tokens": 2})
            assert r.status == 400 and "prompt" in (await r.json())["error"]
            r = await c.post("/chat", data=b"{bad")
            assert r.status == 400
            assert (await c.get("/health")).status == 200
            m = await (await c.get("/metrics")).text()
            assert 'llm_requests_total{status="ok"} 2.0' in m
            assert "llm_completion_tokens_total" in m

    asyncio.run(go())
