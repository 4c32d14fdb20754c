"""Asyncio front for the engine: a dedicated engine thread runs the step loop, HTTP
handlers submit requests and await streamed outputs.

Mirrors the reference's use of ``AsyncLLMEngine.generate`` (an async generator yielding
one output per engine step; llm/serve_llm.py:527-580).  Requests are handed to the
engine thread through a lock-free deque so the event loop never blocks on a running GPU
step; outputs come back with ``loop.call_soon_threadsafe``.

Burst-aware admission: an agent fan-out reaches the backend as N requests
a few ms apart (Agent A's ThreadPoolExecutor, reference agents/agent_a/server.py:534-623);
admitted one by one, the first one's prefill runs alone and the rest queue behind it.  A
request that carries its burst (``burst=(key, size)``: the X-Task-ID and the fan-out width
Agent B forwards as ``x-fanout``) is held until its siblings are in or ``burst_window_s``
has passed since the burst's first arrival, then the whole group is admitted together and
shares ONE prefill forward.  Requests without burst information are never delayed.  TTFT
still runs from each request's arrival, hold time included.  The window also closes early
once ``burst_gap_s`` has passed since the burst's LATEST arrival: a LAN fan-out lands its
siblings well inside that gap, while under arrival skew (netem delay / jitter on the agents,
scripts/traffic/apply_network_emulation.sh) a lone early request is not held for siblings
that are still tens of ms away - it goes ahead alone and the stragglers join the running
batch on arrival.

Watchdog: ``heartbeat`` is refreshed every loop iteration;
``stalled(threshold)`` is true when work is pending but the loop has not progressed for
``threshold`` seconds, and the HTTP layer reports that on /health as 503.
"""
from __future__ import annotations

import asyncio
import collections
import threading
import time
import traceback

from .llm_engine import LLMEngine, RequestOutput
from .sequence import SamplingParams


class EngineDeadError(RuntimeError):
    pass


class AsyncEngine:
    # a flushed burst's record of expected stragglers lives this long
    FLUSHED_TTL_S = 2.0

    def __init__(self, engine: LLMEngine, on_step=None, stream_interval_s: float = 0.05,
                 burst_window_s: float | None = None, burst_gap_s: float | None = None):
        self.engine = engine
        if burst_window_s is None:
            burst_window_s = getattr(engine.cfg, "burst_window_ms", 0.0) / 1000.0
        if burst_gap_s is None:
            burst_gap_s = getattr(engine.cfg, "burst_gap_ms", 4.0) / 1000.0
        self.burst_window_s = max(0.0, float(burst_window_s))
        self.burst_gap_s = max(0.0, float(burst_gap_s))
        # held bursts: key -> [deadline, expected size, [pending entries in arrival order],
        # window deadline (first arrival + window)]
        self._held: dict[str, list] = {}
        # bursts flushed at their deadline: key -> [stragglers still expected, expiry]; a
        # late sibling is admitted at once instead of opening a new window
        self._flushed: dict[str, list] = {}
        self.bursts_coalesced = 0  # groups admitted together (complete or at the deadline)
        # request id -> seconds its burst held it (popped by the server into its records)
        self.hold_s: dict[str, float] = {}
        self.on_step = on_step
        # intermediate outputs of a request are coalesced to at most one per interval (the
        # first token and the final output always go out at once): every delivery wakes the
        # event-loop thread, and a wake-up per request per decode step competes with the
        # engine thread for the GIL (measured: 16 % of the HTTP fan-out throughput)
        self.stream_interval_s = stream_interval_s
        self._last_sent: dict[str, float] = {}
        self._pending: collections.deque = collections.deque()
        self._aborts: collections.deque = collections.deque()
        self._streams: dict[str, tuple] = {}
        self._wake = threading.Event()
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self.heartbeat = time.monotonic()
        self.last_error: str | None = None
        self.fault_injection_delay_s = 0.0  # optional test hook: extra per-step delay

    # ------------------------------------------------------------------------------------
    def start(self):
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name="engine-loop", daemon=True)
            self._thread.start()
        return self

    def shutdown(self):
        self._stop.set()
        self._wake.set()
        if self._thread is not None:
            self._thread.join(timeout=10)
        self.engine.shutdown()

    def stalled(self, threshold_s: float = 60.0) -> bool:
        busy = bool(self._pending) or bool(self._held) or self.engine.has_unfinished()
        return busy and (time.monotonic() - self.heartbeat) > threshold_s

    @property
    def alive(self) -> bool:
        return self._thread is not None and self._thread.is_alive()

    # ------------------------------------------------------------------------------------
    async def generate(self, prompt_ids, sampling: SamplingParams, request_id: str,
                       burst: tuple | None = None):
        """Async generator of cumulative RequestOutputs: the first token at once, then at most
        one per ``stream_interval_s``, and always the final one.  ``burst``: (key, size) of
        the fan-out this request belongs to (burst-aware admission, see the module doc)."""
        if not self.alive:
            raise EngineDeadError("engine loop is not running")
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        self._streams[request_id] = (loop, q)
        self._pending.append((request_id, list(prompt_ids), sampling, time.perf_counter(),
                              burst))
        self._wake.set()
        done = False
        try:
            while True:
                item = await q.get()
                if isinstance(item, BaseException):
                    done = True
                    raise item
                done = item.finished
                yield item
                if done:
                    return
        finally:
            self._streams.pop(request_id, None)
            self._last_sent.pop(request_id, None)
            if not done:  # consumer went away (client disconnect / cancel): free the slot
                self._aborts.append(request_id)
                self._wake.set()

    async def generate_full(self, prompt_ids, sampling: SamplingParams,
                            request_id: str) -> tuple[RequestOutput, float]:
        """Run to completion. Returns (final output, TTFT seconds)."""
        t0 = time.perf_counter()
        ttft = None
        final = None
        async for out in self.generate(prompt_ids, sampling, request_id):
            if ttft is None:
                ttft = time.perf_counter() - t0
            final = out
        return final, (ttft or 0.0)

    # ------------------------------------------------------------------------------------
    def _deliver(self, rid: str, item):
        s = self._streams.get(rid)
        if s is None:
            return
        loop, q = s
        try:
            loop.call_soon_threadsafe(q.put_nowait, item)
        except RuntimeError:  # loop closed
            pass

    def _fail_pending(self, err: BaseException):
        while self._pending:
            self._deliver(self._pending.popleft()[0], err)
        for held in self._held.values():
            for entry in held[2]:
                self._deliver(entry[0], err)
        self._held.clear()

    def _admit(self, entry):
        rid, ids, sp, t_arr = entry[:4]
        try:
            self.engine.add_request(rid, ids, sp, arrival_time=t_arr)
        except Exception as e:  # bad request: fail only that one
            self._deliver(rid, e)

    def _deadline(self, window_end: float, last_arrival: float) -> float:
        if self.burst_gap_s > 0:
            return min(window_end, last_arrival + self.burst_gap_s)
        return window_end

    def _take_pending(self, now: float) -> float | None:
        """Move arrived requests into the engine - bursts held until complete, until the
        window closes, or until no sibling arrived for ``burst_gap_s``.  Returns the earliest
        pending burst deadline (None: nothing held)."""
        for key in [k for k, v in self._flushed.items() if now > v[1]]:
            del self._flushed[key]  # stragglers that never came (failed agent, disconnect)
        while self._pending:
            entry = self._pending.popleft()
            burst = entry[4] if len(entry) > 4 else None
            if not burst or self.burst_window_s <= 0 or int(burst[1]) <= 1:
                self._admit(entry)
                continue
            key, size = str(burst[0]), int(burst[1])
            late = self._flushed.get(key)
            if late is not None:
                late[0] -= 1
                if late[0] <= 0 or now > late[1]:
                    del self._flushed[key]
                self._admit(entry)
                continue
            g = self._held.get(key)
            if g is None:
                g = self._held[key] = [0.0, size, [], entry[3] + self.burst_window_s]
            g[2].append(entry)
            g[0] = self._deadline(g[3], entry[3])
        nearest = None
        for key in list(self._held):
            deadline, size, group = self._held[key][:3]
            if len(group) >= size or now >= deadline:
                del self._held[key]
                if len(group) < size:
                    self._flushed[key] = [size - len(group), now + self.FLUSHED_TTL_S]
                if len(self.hold_s) > 4096:  # callers that never pop: stay bounded
                    self.hold_s.clear()
                for entry in group:  # arrival order: FIFO admission within the burst
                    self.hold_s[entry[0]] = max(0.0, now - entry[3])
                    self._admit(entry)
                self.bursts_coalesced += 1
            elif nearest is None or deadline < nearest:
                nearest = deadline
        return nearest

    def _run(self):
        eng = self.engine
        while not self._stop.is_set():
            self.heartbeat = time.monotonic()
            nearest = self._take_pending(time.perf_counter())
            while self._aborts:
                rid = self._aborts.popleft()
                for key in list(self._held):  # a held request that gave up
                    g = self._held[key][2]
                    g[:] = [e for e in g if e[0] != rid]
                    if not g:
                        del self._held[key]
                eng.abort(rid)
            if not eng.has_unfinished():
                wait = 0.05 if nearest is None else max(0.0, nearest - time.perf_counter())
                self._wake.wait(wait)
                self._wake.clear()
                continue
            try:
                t0 = time.perf_counter()
                outs = eng.step()
                if self.fault_injection_delay_s:
                    time.sleep(self.fault_injection_delay_s)
                if self.on_step is not None and eng.last_step is not None:
                    try:
                        self.on_step(eng.last_step, time.perf_counter() - t0)
                    except Exception:
                        pass
            except Exception as e:
                self.last_error = "".join(traceback.format_exception(e))[-2000:]
                err = RuntimeError(f"engine step failed: {e}")
                # fail every in-flight request; keep the loop alive for new ones
                for s in list(eng.scheduler.running) + list(eng.scheduler.waiting):
                    eng.abort(s.request_id)
                    self._deliver(s.request_id, err)
                dead = eng.dead_ranks() if hasattr(eng, "dead_ranks") else []
                if dead:  # a TP peer is gone: no later step can succeed -> /health 503
                    self.last_error = f"TP ranks {dead} died\n" + self.last_error
                    self._fail_pending(RuntimeError(f"engine dead: TP ranks {dead} died"))
                    return
                if getattr(eng, "step_failure_fatal", False):
                    # TP: rank 0 may already have published this step, so the workers are
                    # inside collectives rank 0 will never join - any later collective would
                    # pair with the wrong step.  Stop the whole TP group; /health -> 503.
                    self.last_error = "TP step failed after publish; engine stopped\n" + \
                        self.last_error
                    self._fail_pending(RuntimeError("engine dead: TP step failed"))
                    try:
                        eng.kill()
                    except Exception:
                        pass
                    return
                continue
            now = time.monotonic()
            for o in outs:
                rid = o.request_id
                if rid not in self._streams:
                    # the consumer already left (disconnect): its generate() popped the
                    # entry; re-adding it here would leak one dict slot per disconnect
                    self._last_sent.pop(rid, None)
                    continue
                last = self._last_sent.get(rid)
                if o.finished or last is None or now - last >= self.stream_interval_s:
                    if o.finished:
                        self._last_sent.pop(rid, None)
                    else:
                        self._last_sent[rid] = now
                    self._deliver(rid, o)
