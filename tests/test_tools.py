"""Tool plane: MCP protocol + demo servers, mcp-tool-db HTTP contract,
OpenAI-compatible proxy, MCP-Universe runner."""
import asyncio
import json
import os
import threading
from pathlib import Path

import httpx
import pytest

from agentic_traffic_testing_amd.experiments import run_mcp_universe
from agentic_traffic_testing_amd.experiments.test_mcp_servers import smoke
from agentic_traffic_testing_amd.tools.mcp_servers import coding_server, finance_server, maps_server
from agentic_traffic_testing_amd.tools.mcp_tool_db import server as tool_db


def _rpc(srv, method, params=None, mid=1):
    return srv.handle({"jsonrpc": "2.0", "id": mid, "method": method, "params": params or {}})


def test_mcp_protocol_in_process():
    srv = maps_server.server
    init = _rpc(srv, "initialize", {"protocolVersion": "2024-11-05"})["result"]
    assert init["serverInfo"]["name"] == "maps-server" and "tools" in init["capabilities"]
    assert _rpc(srv, "notifications/initialized", mid=None) is None
    tools = {t["name"]: t for t in _rpc(srv, "tools/list")["result"]["tools"]}
    assert set(tools) == {"geocode_location", "calculate_distance"}
    assert tools["calculate_distance"]["inputSchema"]["required"] == ["location1", "location2"]
    res = _rpc(srv, "tools/call", {"name": "calculate_distance",
                                   "arguments": {"location1": "Paris, France",
                                                 "location2": "tokyo"}})["result"]
    assert not res["isError"] and res["structuredContent"]["distance_km"] == pytest.approx(9712, abs=5)
    bad = _rpc(srv, "tools/call", {"name": "calculate_distance", "arguments": {"x": 1}})["result"]
    assert bad["isError"]
    assert _rpc(srv, "tools/call", {"name": "nope"})["error"]["code"] == -32602
    assert _rpc(srv, "bogus/method")["error"]["code"] == -32601
    res = _rpc(srv, "resources/read", {"uri": "resource://maps/known-locations"})["result"]
    assert len(json.loads(res["contents"][0]["text"])["locations"]) == 4
    sch = {t["name"]: t for t in _rpc(finance_server.server, "tools/list")["result"]["tools"]}
    assert sch["calculate_portfolio_value"]["inputSchema"]["properties"]["holdings"] == {
        "type": "object", "additionalProperties": {"type": "number"}}


def test_demo_tool_semantics():
    assert maps_server.geocode_location("Atlantis")["found"] is False
    assert maps_server.calculate_distance("London", "Atlantis") == {
        "error": "One or both locations could not be resolved."}
    q = finance_server.get_stock_price("msft")
    assert q["symbol"] == "MSFT" and abs(q["price"] - 378.90) <= 5.0 and q["timestamp"].endswith("Z")
    assert finance_server.get_stock_price("XYZ")["available_symbols"] == ["AAPL", "GOOGL", "MSFT", "TSLA"]
    pv = finance_server.calculate_portfolio_value({"aapl": 10, "UNKNOWN": 3})
    assert pv["total_value"] == 1755.0 and len(pv["positions"]) == 1
    st = coding_server.analyze_code_complexity("def f():\n    pass\n\nclass A:\n    pass\n")
    assert st == {"lines_of_code": 5, "non_empty_lines": 4, "function_count": 1, "class_count": 1}
    r = coding_server.execute_python_code("import sys; print(1); sys.exit(3)")
    assert r["stdout"] == "1\n" and r["return_code"] == 3 and r["success"] is False


def test_mcp_stdio_smoke():
    out = asyncio.run(asyncio.wait_for(smoke(verbose=False), 120))
    assert out["tools"]["coding"] == ["execute_python_code", "analyze_code_complexity"]
    assert out["coding.execute_python_code"]["stdout"].startswith("Hello from MCP")
    assert out["finance.get_stock_price"]["symbol"] == "AAPL"
    assert out["maps.calculate_distance"]["distance_km"] == pytest.approx(5570.22, abs=0.01)


def test_tool_db_http(tmp_path, monkeypatch):
    monkeypatch.setenv("TELEMETRY_LOG_DIR", str(tmp_path))
    srv = tool_db.make_server("127.0.0.1", 0)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    base = f"http://127.0.0.1:{srv.server_address[1]}"
    try:
        r = httpx.post(base + "/query", json={"query": "select 1", "task_id": "t-1"})
        assert r.status_code == 200
        assert r.json() == {"records": [{"id": 1, "value": "Echo of 'select 1'"}]}
        assert httpx.post(base + "/other", json={}).status_code == 404
        assert httpx.post(base + "/query", json={"query": ""}).status_code == 400
        assert httpx.post(base + "/query", content=b"{bad").status_code == 400
        httpx.post(base + "/query", json={"query": "q2"})
    finally:
        srv.shutdown()
        srv.server_close()
    lines = [json.loads(x) for f in tmp_path.glob("*_ToolDB.log") for x in f.read_text().splitlines()]
    assert [e["event_type"] for e in lines] == ["tool_request", "tool_response"] * 2
    assert lines[0]["task_id"] == "t-1" and lines[2]["task_id"] == "unknown-task"
    assert lines[0]["tool_call_id"] == lines[1]["tool_call_id"]


def test_openai_proxy():
    from aiohttp import web

    from agentic_traffic_testing_amd.tools.mcp_universe import openai_proxy

    seen = []

    async def fake_chat(request):
        body = await request.json()
        seen.append(body)
        if body["prompt"].endswith("FAIL"):
            return web.json_response({"error": "boom"}, status=500)
        return web.json_response({"output": "hi there",
                                  "meta": {"prompt_tokens": 7, "completion_tokens": 2}})

    async def main():
        be = web.Application()
        be.router.add_post("/chat", fake_chat)
        be_runner = web.AppRunner(be)
        await be_runner.setup()
        site = web.TCPSite(be_runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        px = web.AppRunner(openai_proxy.create_app(f"http://127.0.0.1:{port}/chat"))
        await px.setup()
        psite = web.TCPSite(px, "127.0.0.1", 0)
        await psite.start()
        pport = psite._server.sockets[0].getsockname()[1]
        async with httpx.AsyncClient(base_url=f"http://127.0.0.1:{pport}") as c:
            ok = await c.post("/v1/chat/completions", json={
                "model": "gpt-4o", "max_tokens": "12",
                "messages": [{"role": "system", "content": "be brief"},
                             {"role": "user", "content": [{"type": "text", "text": "hello"}]}]})
            fail = await c.post("/v1/chat/completions",
                                json={"messages": [{"role": "user", "content": "FAIL"}]})
            bad = await c.post("/v1/chat/completions", json={"messages": []})
            health = await c.get("/health")
        await px.cleanup()
        await be_runner.cleanup()
        return ok, fail, bad, health

    ok, fail, bad, health = asyncio.run(main())
    assert seen[0] == {"prompt": "[SYSTEM]\nbe brief\n\n[USER]\nhello", "max_tokens": 12}
    j = ok.json()
    assert j["object"] == "chat.completion" and j["model"] == "gpt-4o"
    assert j["choices"][0]["message"] == {"role": "assistant", "content": "hi there"}
    assert j["usage"] == {"prompt_tokens": 7, "completion_tokens": 2, "total_tokens": 9}
    assert fail.status_code == 502 and fail.json()["status"] == 500
    assert bad.status_code == 400
    assert health.json()["status"] == "ok"


def test_mcp_universe_runner(tmp_path, capsys):
    bench = tmp_path / "tests" / "benchmark" / "mcpuniverse"
    bench.mkdir(parents=True)
    (bench / "test_benchmark_dummy.py").write_text("print('dummy ok')\n")
    (bench / "test_benchmark_broken.py").write_text("raise SystemExit(2)\n")
    root = str(tmp_path)
    assert run_mcp_universe.main(["--list", "--mcp-universe-dir", root]) == 0
    assert "dummy" in capsys.readouterr().out
    assert run_mcp_universe.main(["dummy", "--mcp-universe-dir", root]) == 0
    assert run_mcp_universe.main(["--all", "--mcp-universe-dir", root]) == 1
    assert run_mcp_universe.main(["nope", "--mcp-universe-dir", root]) == 1
    assert run_mcp_universe.main(["dummy", "--mcp-universe-dir", str(tmp_path / "missing")]) == 1
