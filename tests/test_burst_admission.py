"""Burst-aware admission: fan-out requests that announce their burst
(X-Task-ID + x-fanout) are held until every sibling arrived - or the window expired - and
then share one prefill step; requests without burst information are never delayed."""
import asyncio
import time

from agentic_traffic_testing_amd.config import EngineConfig
from agentic_traffic_testing_amd.engine.async_engine import AsyncEngine
from agentic_traffic_testing_amd.engine.llm_engine import LLMEngine
from agentic_traffic_testing_amd.engine.sequence import SamplingParams


def _engine():
    return LLMEngine(EngineConfig(model="tiny", device="cpu", max_model_len=256,
                                  num_kv_blocks=64, max_num_batched_tokens=256, max_num_seqs=8,
                                  use_graphs=False))


def _run(window_s, plan, gap_s=10.0):
    """plan: [(delay_s, request_id, burst)] submitted in order; returns (steps, ttfts).
    gap_s: the early-close gap (default: large, i.e. the window alone decides)."""
    steps = []
    ae = AsyncEngine(_engine(), on_step=lambda st, dt: steps.append(st),
                     burst_window_s=window_s, burst_gap_s=gap_s).start()
    sp = SamplingParams(temperature=0.0, max_tokens=2, ignore_eos=True)
    ttft = {}

    async def one(delay, rid, burst):
        await asyncio.sleep(delay)
        t0 = time.perf_counter()
        async for out in ae.generate([300 + len(rid), 301, 302, 303, 304], sp, rid, burst=burst):
            ttft.setdefault(rid, time.perf_counter() - t0)

    async def main():
        await asyncio.gather(*(one(*p) for p in plan))

    try:
        asyncio.run(main())
    finally:
        ae._stop.set()
    return steps, ttft, ae


def test_complete_burst_shares_one_prefill():
    plan = [(0.0, "a0", ("task-1", 3)), (0.01, "a1", ("task-1", 3)),
            (0.02, "a2", ("task-1", 3))]
    steps, ttft, ae = _run(0.5, plan)
    first = steps[0]
    assert first.num_seqs == 3 and first.num_decode == 0, steps[:3]
    assert ae.bursts_coalesced == 1
    # released as soon as the last sibling arrived, long before the 0.5 s window
    assert ttft["a2"] < 0.25, ttft


def test_partial_burst_released_at_deadline():
    plan = [(0.0, "b0", ("task-2", 3)), (0.005, "b1", ("task-2", 3))]
    steps, ttft, ae = _run(0.08, plan)
    assert steps[0].num_seqs == 2 and steps[0].num_decode == 0
    assert ttft["b0"] >= 0.07  # held for the window: the third sibling never came


def test_requests_without_burst_are_not_held():
    plan = [(0.0, "c0", None), (0.0, "c1", ("task-3", 1))]
    steps, ttft, ae = _run(1.0, plan)
    assert max(ttft.values()) < 0.5, ttft  # a 1 s window would show
    assert ae.bursts_coalesced == 0


def test_burst_window_zero_disables_holding():
    plan = [(0.0, "d0", ("task-4", 5))]
    steps, ttft, ae = _run(0.0, plan)
    assert ttft["d0"] < 0.5


def test_straggler_after_deadline_not_held_again():
    """A sibling arriving after its burst was flushed at the deadline is admitted at once."""
    # a 250 ms window keeps "held again" (>= 0.25 s) far from a loaded CPU's step time
    plan = [(0.0, "e0", ("task-5", 2)), (0.6, "e1", ("task-5", 2))]
    steps, ttft, ae = _run(0.25, plan)
    assert ttft["e0"] >= 0.2, ttft  # the first one was held for the window
    assert ttft["e1"] < 0.15, ttft  # no second window


# ---- deterministic policy tests on _take_pending (no engine thread, controlled clock) -----
class _FakeEngine:
    class cfg:
        burst_window_ms = 10.0
        burst_gap_ms = 4.0

    def __init__(self):
        self.admitted = []

    def add_request(self, rid, ids, sp, arrival_time=None):
        self.admitted.append(rid)


def _policy(window_s=0.010, gap_s=0.004):
    eng = _FakeEngine()
    return AsyncEngine(eng, burst_window_s=window_s, burst_gap_s=gap_s), eng


def _arrive(ae, rid, t, key="task", size=5):
    ae._pending.append((rid, [1, 2], None, t, (key, size)))


def test_skewed_arrivals_close_window_early():
    """Arrival skew larger than the window (netem-like, 30 ms apart): the lone early request
    waits only the 4 ms gap, not the 10 ms window, and every later sibling goes at once."""
    ae, eng = _policy()
    t0 = 100.0
    _arrive(ae, "s0", t0)
    assert ae._take_pending(t0) == t0 + 0.004  # held, deadline = last arrival + gap
    assert eng.admitted == []
    ae._take_pending(t0 + 0.0041)
    assert eng.admitted == ["s0"]
    for i in range(1, 5):  # stragglers of the flushed burst: admitted on arrival
        t = t0 + 0.030 * i
        _arrive(ae, f"s{i}", t)
        ae._take_pending(t)
        assert eng.admitted[-1] == f"s{i}"
    assert not ae._held and not ae._flushed


def test_lan_burst_coalesces_within_gap():
    """A LAN fan-out (siblings 0.5-1 ms apart) is held to the last sibling and admitted as
    one group; each arrival pushes the gap deadline, the window caps it."""
    ae, eng = _policy()
    t0 = 5.0
    for i in range(5):
        _arrive(ae, f"l{i}", t0 + 0.0008 * i)
        dl = ae._take_pending(t0 + 0.0008 * i)
        if i < 4:
            assert eng.admitted == [] and abs(dl - (t0 + 0.0008 * i + 0.004)) < 1e-9
    assert eng.admitted == [f"l{i}" for i in range(5)]
    assert ae.bursts_coalesced == 1


def test_window_caps_a_slow_trickle():
    ae, eng = _policy(window_s=0.010, gap_s=0.004)
    t0 = 1.0
    for i in range(4):  # 3 ms apart: the gap never expires, the 10 ms window does
        _arrive(ae, f"w{i}", t0 + 0.003 * i)
        ae._take_pending(t0 + 0.003 * i)
    assert eng.admitted == []
    assert ae._take_pending(t0 + 0.0095) == t0 + 0.010
    ae._take_pending(t0 + 0.0101)
    assert eng.admitted == ["w0", "w1", "w2", "w3"]


def test_flushed_records_expire_without_stragglers():
    """A burst flushed at its deadline whose siblings never come must not leak its record
    (the dict grew without bound in a long-running server)."""
    ae, eng = _policy()
    for k in range(50):
        t = 10.0 + k * 0.1
        _arrive(ae, f"f{k}", t, key=f"task-{k}", size=3)
        ae._take_pending(t)
        ae._take_pending(t + 0.005)  # gap expired: flushed with 2 stragglers expected
    assert len(eng.admitted) == 50
    assert 0 < len(ae._flushed) <= 50
    ae._take_pending(10.0 + 50 * 0.1 + ae.FLUSHED_TTL_S + 0.01)
    assert ae._flushed == {}
