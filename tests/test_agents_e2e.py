"""Full L5-L8 request flow on CPU: real LLM backend (tiny engine) + 5 Agent B + Agent A over
HTTP on 127.0.0.1.  Checks the JSON contracts, SSE events, persistence,
telemetry / llm_calls logs and trace propagation."""
import json
import os

import httpx
import pytest

from agentic_traffic_testing_amd.testing.stack import Stack, cpu_engine


@pytest.fixture(scope="module")
def stack(tmp_path_factory):
    d = tmp_path_factory.mktemp("logs")
    eng = cpu_engine(max_model_len=2048, num_kv_blocks=1024, max_num_batched_tokens=2048)
    env = {"LLM_MAX_TOKENS": "8", "LLM_MAX_MODEL_LEN": "2048", "AGENTVERSE_ORACLE": "1",
           "NODE_NAME": "testnode"}
    s = Stack(eng, n_agent_b=5, log_dir=str(d), env=env)
    s.llm.state.s.max_tokens = 8
    yield s
    s.stop()


def test_llm_backend_contract(stack):
    url = stack.llm.url
    assert httpx.get(url + "/health").json() == {"status": "ok"}
    r = httpx.post(url + "/chat", json={"prompt": "hello there", "max_tokens": 5},
                   headers={"X-Request-ID": "abc123"}, timeout=60)
    assert r.status_code == 200
    body = r.json()
    assert set(body) == {"output", "meta"}
    m = body["meta"]
    for k in ("request_id", "latency_ms", "queue_wait_s", "prompt_tokens", "completion_tokens",
              "total_tokens", "otel"):
        assert k in m
    assert m["request_id"] == "abc123" and m["completion_tokens"] == 5
    assert m["total_tokens"] == m["prompt_tokens"] + 5
    assert httpx.post(url + "/chat", content=b"{nope").status_code == 400
    assert httpx.post(url + "/chat", json={"max_tokens": 3}).json() == {
        "error": "Missing 'prompt' field"}
    # aliases + input field
    assert httpx.post(url + "/generate", json={"input": "x", "max_tokens": 2},
                      timeout=60).status_code == 200
    text = httpx.get(url + "/metrics").text
    for name in ("llm_requests_total", "llm_request_latency_seconds_bucket",
                 "llm_queue_wait_seconds_bucket", "llm_inflight_requests",
                 "llm_prompt_tokens_total", "llm_completion_tokens_total",
                 "llm_batch_size_bucket", "llm_config_max_num_seqs",
                 "llm_kv_cache_num_gpu_blocks", "llm_computed_max_concurrency",
                 "llm_interarrival_seconds_bucket", "llm_ttft_seconds_bucket"):
        assert name in text, name
    assert 'le="0.5"' in text and 'le="180.0"' in text


def test_task_scenarios(stack):
    a = stack.agent_a_url
    r = httpx.post(a + "/task", json={"task": "Add 2 and 3", "scenario": "agentic_simple"},
                   timeout=120).json()
    assert r["agent_id"] == "AgentA" and r["total_llm_calls"] == 1
    keys = {"task_id", "agent_id", "scenario", "task_query", "task_start", "task_end",
            "total_llm_calls", "total_prompt_tokens", "total_completion_tokens", "total_tokens",
            "total_latency_ms", "llm_latency_ms", "total_agent_hops", "cost_estimate_usd",
            "output", "agent_b_output", "agent_b_outputs", "agent_a_progress_notes",
            "llm_requests"}
    assert keys <= set(r)

    r = httpx.post(a + "/task", json={"task": "Plan a trip", "scenario": "agentic_parallel",
                                      "agent_count": 5}, timeout=180).json()
    # planning + 5 workers + final
    assert r["total_llm_calls"] == 7 and r["total_agent_hops"] == 5
    assert len(r["agent_b_outputs"]) == 5
    assert {o["agent_index"] for o in r["agent_b_outputs"]} == {1, 2, 3, 4, 5}
    # fan-out hit 5 different Agent B replicas
    assert len({o["endpoint"] for o in r["agent_b_outputs"]}) == 5

    r = httpx.post(a + "/task", json={"task": "Write a poem", "scenario": "agentic_multi_hop",
                                      "max_agent_turns": 2}, timeout=180).json()
    assert r["total_llm_calls"] == 2 * 2 + 1
    assert len(r["agent_a_progress_notes"]) == 2


def test_agentverse_json_and_persistence(stack):
    a = stack.agent_a_url
    r = httpx.post(a + "/agentverse", json={"task": "Design a calculator",
                                            "max_iterations": 2, "success_threshold": 101},
                   timeout=600)
    assert r.status_code == 200
    res = r.json()
    for k in ("task_id", "original_task", "completed", "iterations", "duration_seconds",
              "final_output", "stages", "iteration_history", "llm_requests"):
        assert k in res
    assert set(res["stages"]) == {"recruitment", "decision", "execution", "evaluation"}
    assert res["completed"] is True
    seqs = [q["seq"] for q in res["llm_requests"]]
    assert seqs == list(range(1, len(seqs) + 1))  # unique, ordered under parallel fan-out
    # oracle mode recruits 3..5 experts
    assert 3 <= len(res["stages"]["recruitment"]["experts"]) <= 5
    g = httpx.get(f"{a}/agentverse/{res['task_id']}").json()
    assert g["task_id"] == res["task_id"] and g["result"]["task_id"] == res["task_id"]
    g2 = httpx.get(f"{a}/agentverse?taskId={res['task_id']}").json()
    assert g2["task_id"] == res["task_id"]
    assert httpx.get(f"{a}/agentverse/does-not-exist").status_code == 404
    assert httpx.get(f"{a}/agentverse/bad..id").status_code == 400


def test_agentverse_sse(stack):
    a = stack.agent_a_url
    events = []
    with httpx.stream("POST", a + "/agentverse", json={"task": "Summarise quantum computing",
                                                       "max_iterations": 1, "stream": True},
                      timeout=600) as r:
        ev = None
        for line in r.iter_lines():
            if line.startswith("event: "):
                ev = line[7:]
            elif line.startswith("data: ") and ev:
                events.append((ev, json.loads(line[6:])))
    names = [e for e, _ in events]
    assert names[0] == "iteration_start" and names[-1] == "complete"
    for n in ("stage_start", "stage_complete", "llm_request", "execution_result",
              "iteration_complete"):
        assert n in names


def test_logs_written(stack):
    d = stack.log_dir
    calls = [json.loads(line) for line in open(os.path.join(d, "llm_calls.jsonl"))]
    assert calls and {"call_id", "task_id", "agent_id", "call_type", "latency_ms",
                      "http_status"} <= set(calls[0])
    tele = [f for f in os.listdir(d) if f.endswith(".log")]
    assert any("AgentA" in f for f in tele) and any("AgentB" in f for f in tele)
    ev = [json.loads(line) for line in open(os.path.join(d, "testnode_AgentB.log"))]
    assert {"task_id", "agent_id", "tool_call_id", "event_type", "message", "timestamp_ms",
            "scenario", "extra", "node_id"} <= set(ev[0])


def test_trace_propagation(stack):
    tp = "00-0af7651916cd43dd8448eb211c80319c-b7ad6b7169203331-01"
    r = httpx.post(stack.llm.url + "/chat", json={"prompt": "trace me", "max_tokens": 2},
                   headers={"traceparent": tp}, timeout=60).json()
    assert r["meta"]["otel"]["trace_id"] == "0af7651916cd43dd8448eb211c80319c"


def test_engine_child_spans(stack, monkeypatch):
    """engine.prefill (under llm.time_to_first_token) and engine.decode_step (under
    llm.generate) are emitted per request with the engine's own timestamps."""
    from agentic_traffic_testing_amd.utils import otel

    spans = []

    class Sink:
        def submit(self, sp):
            spans.append(sp)

    monkeypatch.setattr(otel, "_exporter", lambda: Sink())
    tp = "00-1af7651916cd43dd8448eb211c80319c-b7ad6b7169203331-01"
    r = httpx.post(stack.llm.url + "/chat", json={"prompt": "spans please", "max_tokens": 5},
                   headers={"traceparent": tp}, timeout=60)
    assert r.status_code == 200
    by = {s.name: s for s in spans}
    for name in ("llm.time_to_first_token", "llm.generate", "engine.prefill",
                 "engine.decode_step"):
        assert name in by, sorted(by)
    pre, dec = by["engine.prefill"], by["engine.decode_step"]
    assert pre.parent.span_id == by["llm.time_to_first_token"].get_span_context().span_id
    assert dec.parent.span_id == by["llm.generate"].get_span_context().span_id
    assert pre.get_span_context().trace_id == 0x1af7651916cd43dd8448eb211c80319c
    assert pre.start_ns <= pre.end_ns <= dec.start_ns <= dec.end_ns
    assert dec.attributes["engine.decode_steps"] == 4
