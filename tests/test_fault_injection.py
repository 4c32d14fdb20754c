"""Failure detection and fault injection on the real CPU HTTP stack.

* ``LLM_FAULT_FAIL_RATE`` / ``LLM_FAULT_DELAY_MS`` make the LLM backend fail or delay
  requests, which is what exercises the agents' error paths (Agent A answers 502).
* The engine watchdog: a stalled engine loop turns ``/health`` into 503.
"""
import time

import httpx
import pytest

from agentic_traffic_testing_amd.testing.stack import Stack, cpu_engine


@pytest.fixture(scope="module")
def stack(tmp_path_factory):
    d = tmp_path_factory.mktemp("logs")
    eng = cpu_engine(max_model_len=1024, num_kv_blocks=256, max_num_batched_tokens=1024)
    s = Stack(eng, n_agent_b=2, log_dir=str(d), env={"LLM_MAX_TOKENS": "4"})
    s.llm.state.s.max_tokens = 4
    yield s
    s.stop()


def test_injected_failures_reach_the_agents(stack):
    s = stack.llm.state.s
    try:
        s.fault_fail_rate = 1.0
        r = httpx.post(stack.llm.url + "/chat", json={"prompt": "x", "max_tokens": 2}, timeout=60)
        assert r.status_code == 500 and "injected fault" in r.json()["error"]
        r = httpx.post(stack.agent_a_url + "/task",
                       json={"task": "Add 2 and 3", "scenario": "agentic_simple"}, timeout=120)
        assert r.status_code == 502
    finally:
        s.fault_fail_rate = 0.0
    assert 'status="error"' in httpx.get(stack.llm.url + "/metrics").text
    r = httpx.post(stack.llm.url + "/chat", json={"prompt": "x", "max_tokens": 2}, timeout=60)
    assert r.status_code == 200


def test_injected_delay(stack):
    s = stack.llm.state.s
    try:
        s.fault_delay_s = 0.3
        r = httpx.post(stack.llm.url + "/chat", json={"prompt": "x", "max_tokens": 2}, timeout=60)
        assert r.status_code == 200 and r.json()["meta"]["latency_ms"] >= 300
    finally:
        s.fault_delay_s = 0.0


def test_watchdog_reports_stalled_engine(stack):
    """A per-step delay longer than the watchdog threshold makes /health 503 while work is
    pending, and healthy again once the loop progresses."""
    s, ae = stack.llm.state.s, stack.llm.aengine
    old = s.watchdog_s
    try:
        s.watchdog_s = 0.2
        ae.fault_injection_delay_s = 1.5
        with httpx.Client(timeout=60) as c:
            import threading

            t = threading.Thread(target=lambda: c.post(stack.llm.url + "/chat",
                                                       json={"prompt": "x", "max_tokens": 3}))
            t.start()
            deadline = time.time() + 10
            seen = False
            while time.time() < deadline and not seen:
                seen = httpx.get(stack.llm.url + "/health").status_code == 503
                time.sleep(0.05)
            assert seen, "watchdog never reported the stalled loop"
            ae.fault_injection_delay_s = 0.0
            t.join(60)
        s.watchdog_s = old
        assert httpx.get(stack.llm.url + "/health").status_code == 200
    finally:
        s.watchdog_s = old
        ae.fault_injection_delay_s = 0.0
