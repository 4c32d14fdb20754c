"""Static UI: JS parses, the SSE parser handles the backend's framing,
and the dev server serves pages + templates."""
import importlib.util
import json
import shutil
import subprocess
import threading
from pathlib import Path

import httpx
import pytest

UI = Path(__file__).resolve().parents[1] / "ui"


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_js_syntax_and_sse_parser():
    for f in sorted((UI / "agentverse" / "js").glob("*.js")):
        r = subprocess.run(["node", "--check", str(f)], capture_output=True, text=True)
        assert r.returncode == 0, (f, r.stderr)
    script = (UI / "agentverse/js/utils.js").read_text() + (UI / "agentverse/js/streaming.js").read_text() + """
const a = parseSseBlock('event: stage_start\\ndata: {"stage":"recruitment","iteration":1}');
const b = parseSseBlock('data: not json');
const c = parseSseBlock('event: ping');
console.log(JSON.stringify([a, b, c, U.baseOf('http://h:8101/agentverse'), U.hostOf('http://x:1/y')]));
"""
    r = subprocess.run(["node", "-e", script], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    a, b, c, base, host = json.loads(r.stdout)
    assert a == {"event": "stage_start", "data": {"stage": "recruitment", "iteration": 1}}
    assert b == {"event": "message", "data": "not json"} and c is None
    assert base == "http://h:8101" and host == "x:1"


def test_sse_framing_matches_agent_a():
    """The SSE writer used by Agent A emits exactly the frames the UI parser expects."""
    from agentic_traffic_testing_amd.agents.common.http import JsonHandler

    class Capture:
        def __init__(self):
            self.buf = b""

        def write(self, b):
            self.buf += b

        def flush(self):
            pass

    h = JsonHandler.__new__(JsonHandler)
    h.wfile = Capture()
    h.send_sse("stage_complete", {"stage": "evaluation", "score": 95})
    assert h.wfile.buf.decode() == 'event: stage_complete\ndata: {"stage": "evaluation", "score": 95}\n\n'


def test_ui_dev_server():
    spec = importlib.util.spec_from_file_location("ui_serve", UI / "serve.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    srv = mod.make_server("127.0.0.1", 0)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    base = f"http://127.0.0.1:{srv.server_address[1]}"
    try:
        assert "AgentVerse" in httpx.get(base + "/").text
        assert 'id="agent_b_workers"' not in httpx.get(base + "/chat/").text
        assert "agent_b_workers" in httpx.get(base + "/chat/").text
        assert httpx.get(base + "/agentverse/js/streaming.js").status_code == 200
        wf = httpx.get(base + "/agentverse/templates/agentverse_workflow.json").json()
        assert len(wf["example_tasks"]) == 4
        t = httpx.get(base + "/chat/templates/mas_agent_contracts_simple.json").json()
        assert t["ui_defaults"]["scenario"] == "agentic_parallel"
    finally:
        srv.shutdown()
        srv.server_close()
