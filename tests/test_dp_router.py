"""Data-parallel router over two real CPU backends."""
import asyncio
import threading

import httpx
import pytest
from aiohttp import web

from agentic_traffic_testing_amd.parallel.dp_router import Router, create_app
from agentic_traffic_testing_amd.testing.stack import LLMBackendThread, cpu_engine


class RouterThread:
    def __init__(self, router):
        self.loop = asyncio.new_event_loop()
        self.ready = threading.Event()
        self.router = router
        threading.Thread(target=self._run, daemon=True).start()
        assert self.ready.wait(30)

    def _run(self):
        asyncio.set_event_loop(self.loop)
        self.runner = web.AppRunner(create_app(self.router, probe_interval_s=0.2))
        self.loop.run_until_complete(self.runner.setup())
        site = web.TCPSite(self.runner, "127.0.0.1", 0)
        self.loop.run_until_complete(site.start())
        self.url = f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}"
        self.ready.set()
        self.loop.run_forever()

    def stop(self):
        asyncio.run_coroutine_threadsafe(self.runner.cleanup(), self.loop).result(10)
        self.loop.call_soon_threadsafe(self.loop.stop)


@pytest.fixture(scope="module")
def backends():
    bs = [LLMBackendThread(cpu_engine(max_model_len=512, num_kv_blocks=128,
                                      max_num_batched_tokens=512)) for _ in range(2)]
    for b in bs:
        b.state.s.max_tokens = 4
    yield bs
    for b in bs:
        b.stop()


def test_router_balances_and_records_metrics(backends):
    rt = RouterThread(Router([b.url for b in backends], "least_loaded"))
    try:
        def one(i):
            return httpx.post(rt.url + "/chat", json={"prompt": f"hello {i}", "max_tokens": 3},
                              headers={"X-Request-ID": f"r{i}"}, timeout=120)
        import concurrent.futures as cf
        with cf.ThreadPoolExecutor(6) as ex:
            rs = list(ex.map(one, range(6)))
        assert all(r.status_code == 200 for r in rs)
        assert rs[0].json()["meta"]["request_id"] == "r0"
        served = [r.requests for r in rt.router.replicas]
        assert sum(served) == 6 and min(served) >= 1
        m = httpx.get(rt.url + "/metrics").text
        assert 'llm_requests_total{status="success"} 6.0' in m
        assert "llm_router_replica_inflight" in m and "llm_ttft_seconds_bucket" in m
        assert httpx.post(rt.url + "/chat", json={"max_tokens": 3}).status_code == 400
        assert httpx.get(rt.url + "/health").json()["status"] == "ok"
    finally:
        rt.stop()


def test_router_task_affinity_and_failover(backends):
    router = Router([b.url for b in backends] + ["http://127.0.0.1:9"], "task_affinity")
    rt = RouterThread(router)
    try:
        import time
        time.sleep(0.6)  # probe marks the dead replica unhealthy
        assert not router.replicas[2].healthy
        for _ in range(3):
            r = httpx.post(rt.url + "/chat", json={"prompt": "same task", "max_tokens": 2},
                           headers={"X-Task-ID": "task-42"}, timeout=120)
            assert r.status_code == 200
        counts = [rep.requests for rep in router.replicas]
        assert sorted(counts) == [0, 0, 3]  # all three on one live replica
    finally:
        rt.stop()


@pytest.mark.gpu
def test_router_two_gpu_replicas_one_gpu(tmp_path):
    """Two serve_llm replica PROCESSES (the spawn_replicas path of a multi-GPU node, both
    pinned to GPU 0 here) behind the router: concurrent /chat requests are answered by real
    HIP engines and spread over both replicas; /health and the contract metrics work."""
    import socket
    import time

    from agentic_traffic_testing_amd.parallel.dp_router import spawn_replicas

    with socket.socket() as s0:
        s0.bind(("127.0.0.1", 0))
        base = s0.getsockname()[1]
    args = ["--model", "small", "--max-model-len", "512", "--gpu-memory-utilization", "0.2",
            "--max-num-seqs", "4"]
    procs = spawn_replicas(2, base, args, log_dir=str(tmp_path), gpus=[0, 0])
    rt = None
    try:
        urls = [f"http://127.0.0.1:{base + i}" for i in range(2)]
        t0 = time.time()
        for u in urls:
            while True:
                assert all(p.poll() is None for p in procs), open(
                    tmp_path / "llm_replica_0.log").read()[-2000:]
                try:
                    if httpx.get(u + "/health", timeout=2).status_code == 200:
                        break
                except httpx.HTTPError:
                    pass
                assert time.time() - t0 < 240, "replicas did not come up"
                time.sleep(1)
        rt = RouterThread(Router(urls, "round_robin"))
        import concurrent.futures as cf

        def call(i):
            r = httpx.post(rt.url + "/chat", json={"prompt": f"hello {i}", "max_tokens": 8},
                           timeout=120)
            r.raise_for_status()
            return r.json()

        with cf.ThreadPoolExecutor(6) as ex:
            outs = list(ex.map(call, range(6)))
        assert all(o["meta"]["completion_tokens"] > 0 for o in outs)
        assert all(rep.requests >= 2 for rep in rt.router.replicas)
        assert httpx.get(rt.url + "/health", timeout=5).status_code == 200
        m = httpx.get(rt.url + "/metrics", timeout=5).text
        assert "llm_requests_total" in m
    finally:
        if rt is not None:
            rt.stop()
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(30)
            except Exception:
                p.kill()
