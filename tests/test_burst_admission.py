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


def _run(window_s, plan):
    """plan: [(delay_s, request_id, burst)] submitted in order; returns (steps, ttfts)."""
    steps = []
    ae = AsyncEngine(_engine(), on_step=lambda st, dt: steps.append(st),
                     burst_window_s=window_s).start()
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
    plan = [(0.0, "e0", ("task-5", 2)), (0.3, "e1", ("task-5", 2))]
    steps, ttft, ae = _run(0.05, plan)
    assert ttft["e1"] < 0.04, ttft  # no second 50 ms window
