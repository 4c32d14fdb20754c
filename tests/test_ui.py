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


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_agentverse_state_reducer_on_recorded_sse():
    """the SPA's run reducer (ui-state.js) and iteration diff (diff.js) over a
    recorded SSE stream of real AgentVerse runs (tests/fixtures/agentverse_sse.txt, captured
    from the in-process stack: a horizontal and a vertical iteration, every orchestrator
    event type) plus
    the client-side events (llm_error, workflow_error, cancelled, error, fallback)."""
    js = UI / "agentverse" / "js"
    fixture = Path(__file__).resolve().parent / "fixtures" / "agentverse_sse.txt"
    script = "\n".join((js / f).read_text() for f in ("utils.js", "streaming.js", "diff.js")) + \
        "\n" + (js / "ui-state.js").read_text() + r"""
const fs = require('fs');
const text = fs.readFileSync(process.argv[1], 'utf8');
const runs = [];
let run = newRun('t');
const kinds = new Set();
for (const block of text.split('\n\n')) {
  const ev = parseSseBlock(block);
  if (!ev) continue;
  kinds.add(ev.event);
  applyRunEvent(run, ev.event, ev.data);
  if (ev.event === 'complete') { runs.push(run); run = newRun('t'); }
}
// client-side / failure events on a fresh run
const extra = newRun('x');
applyRunEvent(extra, 'iteration_start', { iteration: 0, max_iterations: 3 });
applyRunEvent(extra, 'stage_start', { stage: 'recruitment', iteration: 0 });
applyRunEvent(extra, 'llm_error', { seq: 1, stage: 'recruitment', error: 'HTTP 502' });
applyRunEvent(extra, 'fallback', { message: 'no SSE' });
applyRunEvent(extra, 'workflow_error', { error: 'backend down' });
applyRunEvent(extra, 'cancelled', {});
const errRun = newRun('e');
applyRunEvent(errRun, 'error', { error: 'HTTP 500' });
const out = runs.map((r) => {
  const its = Object.keys(r.iterations).map(Number).sort((a, b) => a - b);
  const d = its.length > 1 ? Diff.iterations(r.iterations[its[0]], r.iterations[its[1]]) : null;
  return {
    status: r.status, calls: r.llmCalls, resultCalls: (r.result.llm_requests || []).length,
    seqs: r.requests.map((q) => q.seq), iterations: its, resultIterations: r.result.iterations,
    rounds: its.map((i) => r.iterations[i].discussion.length),
    vertical: its.map((i) => r.iterations[i].vertical.length),
    executions: its.map((i) => r.iterations[i].executions.length),
    facts: its.map((i) => Diff.facts(r.iterations[i])),
    diff: d, stagesDone: Object.keys(r.stages).filter((k) => r.stages[k].state === 'done').sort(),
  };
});
console.log(JSON.stringify({ kinds: Array.from(kinds).sort(), runs: out,
  extra: { status: extra.status, errors: extra.llmErrors, error: extra.error, stage: extra.stages.recruitment.state },
  err: { status: errRun.status, error: errRun.error },
  lines: Diff.lines('a\nb\nc', 'a\nc\nd'), clock: fmtClock(3725) }));
"""
    r = subprocess.run(["node", "-e", script, str(fixture)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert set(d["kinds"]) >= {"iteration_start", "stage_start", "stage_complete", "llm_request",
                               "discussion_round", "vertical_iteration", "execution_result",
                               "iteration_complete", "complete"}
    assert len(d["runs"]) >= 1
    for run in d["runs"]:
        assert run["status"] in ("done", "incomplete")
        assert run["calls"] == run["resultCalls"] > 0
        assert run["seqs"] == sorted(set(run["seqs"]))  # one entry per call, seq order
        assert run["iterations"][-1] == run["resultIterations"]
        assert all(n > 0 for n in run["executions"])
        assert all(f["experts"] and f["score"] is not None for f in run["facts"])
        assert {"recruitment", "decision", "execution", "evaluation", "synthesis"} <= set(run["stagesDone"])
        if run["diff"]:
            assert set(run["diff"]) >= {"experts", "structure", "score", "criteria", "decision"}
            assert run["diff"]["score"]["delta"] == run["facts"][1]["score"] - run["facts"][0]["score"]
    # horizontal discussion rounds and vertical review iterations both reach their snapshots
    assert any(sum(r["rounds"]) for r in d["runs"]) and any(sum(r["vertical"]) for r in d["runs"])
    assert d["extra"] == {"status": "cancelled", "errors": 1, "error": "backend down",
                          "stage": "cancelled"}
    assert d["err"] == {"status": "error", "error": "HTTP 500"}
    assert [x["op"] for x in d["lines"]] == ["=", "-", "=", "+"]
    assert d["clock"] == "1:02:05"
