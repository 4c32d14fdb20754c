"""Synchronous serving engine: scheduler + model runner + stop handling.

The reference drives vLLM's ``AsyncLLMEngine.generate`` (llm/serve_llm.py:504-612); this
engine provides the same contract (prompt in, streamed outputs, TTFT = time to the first
yielded output) on the MI355X-native runner.  ``async_engine.AsyncEngine`` wraps it with
a background step loop for the HTTP front end.
"""
from __future__ import annotations

import random
import threading
import time
from dataclasses import dataclass, field

import numpy as np

from ..config import EngineConfig, resolve_model
from ..utils import roctx
from .model_runner import ModelRunner
from .scheduler import Batch, Scheduler
from .sequence import SamplingParams, Sequence, SeqStatus
from .tokenizer import get_tokenizer

PENDING_TOKEN = -1  # output slot of a launched step whose token the host has not seen yet


@dataclass
class RequestOutput:
    request_id: str
    token_ids: list
    finished: bool
    finish_reason: str | None = None
    prompt_tokens: int = 0
    cached_prompt_tokens: int = 0
    arrival_time: float = 0.0
    first_token_time: float | None = None
    first_scheduled_time: float | None = None
    finish_time: float | None = None
    new_token_ids: list = field(default_factory=list)

    @property
    def completion_tokens(self) -> int:
        return len(self.token_ids)

    @property
    def ttft(self) -> float | None:
        if self.first_token_time is None:
            return None
        return self.first_token_time - self.arrival_time

    @property
    def queue_wait(self) -> float | None:
        if self.first_scheduled_time is None:
            return None
        return self.first_scheduled_time - self.arrival_time


@dataclass
class StepStats:
    num_seqs: int
    num_tokens: int
    num_decode: int
    seconds: float


@dataclass
class _Inflight:
    batch: object
    handle: dict
    marks: list      # (seq, output index of this step's token, num_computed after it)
    t0: float


class LLMEngine:
    def __init__(self, cfg: EngineConfig, runner: ModelRunner | None = None, device=None):
        self.cfg = cfg
        self.model_cfg, weights_dir = resolve_model(cfg.model)
        self.tokenizer = get_tokenizer(weights_dir or cfg.model, self.model_cfg.vocab_size)
        dev = device or cfg.device
        self.runner = runner or ModelRunner(cfg, self.model_cfg, dev, weights_dir=weights_dir)
        self.scheduler = Scheduler(self.runner.bm, cfg.max_num_seqs, cfg.max_num_batched_tokens,
                                   cfg.max_model_len, cfg.long_prefill_token_threshold)
        self.eos_ids = set(self.model_cfg.eos_token_ids) | {self.tokenizer.eos_token_id}
        self.lock = threading.RLock()
        self.last_step: StepStats | None = None
        self.total_steps = 0
        self.total_generated = 0
        self.total_prompt = 0
        self.batch_size_history: list = []
        # host-side step breakdown (seconds): scheduler, runner.execute (prep + GPU + sync),
        # output processing
        self.timing = {"schedule": 0.0, "execute": 0.0, "post": 0.0, "steps": 0,
                       "lookahead_steps": 0}
        self._rng = random.Random(cfg.seed)
        # async look-ahead decode: the step launched but not yet collected (see step())
        self._inflight: _Inflight | None = None
        self._last_collect = 0.0
        # (a TP engine warms up itself once its worker group is fully set up)
        if cfg.startup_warmup and self.runner.is_cuda and not getattr(self, "_defer_warmup",
                                                                      False):
            self.warmup()

    def warmup(self) -> None:
        """Serve throw-away requests of the fan-out workload's step shapes - a 17-row
        planning step, a 5 x 17-row burst (wide kernel), 200 / 600-row prefills (mid-M kernel
        + tuned library GEMMs), a long prefill (library + flash prefill tiles), their decode
        steps and one top-k / top-p sampled request - then drop their prefix-cache entries
        and reset the engine's statistics and request-seed stream.  Every code object those
        paths reach (HIP translation units, PyTorch kernels, library solutions) is then loaded
        before the first real request: bench/coldstart.py measures first vs repeat TTFT per
        shape."""
        r = self.runner
        room = min(self.cfg.max_model_len - 8,
                   r.num_blocks * r.block_size // 2, self.cfg.max_num_batched_tokens * 4)
        vocab = max(8, min(self.model_cfg.vocab_size, 32000))
        rng = np.random.default_rng(0)

        def toks(n):
            return rng.integers(min(1000, vocab // 2), vocab, size=n).tolist()

        greedy = SamplingParams(temperature=0.0, max_tokens=2, ignore_eos=True)
        t0 = time.perf_counter()
        shapes = [[17], [17] * 5] + [[n] for n in (200, 600, 3000) if n <= room]
        for sizes in shapes:
            if sum(sizes) <= room:
                self.generate([toks(n) for n in sizes], greedy)
        self.generate([toks(17)], SamplingParams(temperature=0.7, top_p=0.9, top_k=40,
                                                 max_tokens=2, ignore_eos=True, seed=1))
        r.reset_state()
        self.total_steps = self.total_generated = self.total_prompt = 0
        self.batch_size_history = []
        self.last_step = None
        self.timing = {k: (0 if k.endswith("steps") else 0.0) for k in self.timing}
        self._rng = random.Random(self.cfg.seed)
        self.warmup_seconds = time.perf_counter() - t0

    # ------------------------------------------------------------------------------------
    def add_request(self, request_id: str, prompt_ids, sampling: SamplingParams,
                    arrival_time: float | None = None) -> Sequence:
        ids = list(map(int, prompt_ids))
        if not ids:
            ids = [self.tokenizer.bos_token_id]
        limit = self.cfg.max_model_len - 1
        if len(ids) > limit:
            ids = ids[:limit]
        seq = Sequence(request_id=request_id, prompt_ids=ids, sampling=sampling)
        if arrival_time is not None:
            seq.arrival_time = arrival_time
        seq.seed = sampling.seed if sampling.seed is not None else self._rng.getrandbits(62)
        with self.lock:
            self.scheduler.add(seq)
        return seq

    def abort(self, request_id: str):
        with self.lock:
            self.scheduler.abort(request_id)

    def has_unfinished(self) -> bool:
        return self.scheduler.has_work() or self._inflight is not None

    # ------------------------------------------------------------------------------------
    def step(self) -> list[RequestOutput]:
        """One engine step; returns the outputs it produced.

        Async look-ahead decode (``EngineConfig.async_decode``): a decode-only graph step is
        launched, then - before the host waits for its tokens - the step that continues
        every one of its sequences is launched too, its input tokens taken on the device
        from the first step's samples (``ops.embed`` feed_prev path).  The host's scheduling,
        metadata packing and output processing then overlap the GPU instead of sitting
        between two replays.  Look-ahead stops (one plain step drains it) whenever requests
        are waiting for admission, a sequence finishes by length, or the KV pool is full,
        so outputs are identical to the synchronous engine: a look-ahead token of a sequence
        that stopped on EOS is discarded."""
        with self.lock:
            if self._inflight is None:
                ts = time.perf_counter()
                with roctx.range("engine.schedule"):
                    batch = self.scheduler.schedule()
                if batch.empty:
                    return []
                t0 = time.perf_counter()
                self.timing["schedule"] += t0 - ts
                if not (self.cfg.async_decode and self.runner.launchable(batch)):
                    with roctx.range("engine.sync_step" if batch.num_decode == len(batch.seqs)
                                     else "engine.prefill_step"):
                        return self._sync_step(batch, t0)
                with roctx.range("engine.launch"):
                    self._inflight = self._launch(batch, lookahead=False)
            cur = self._inflight
            nxt = self._lookahead_batch(cur)
            if nxt is not None:
                with roctx.range("engine.launch_lookahead"):
                    self._inflight = self._launch(nxt, lookahead=True)
            else:
                self._inflight = None
            with roctx.range("engine.collect"):
                return self._collect(cur)

    def _launch(self, batch, lookahead: bool) -> "_Inflight":
        t0 = time.perf_counter()
        h = self.runner.launch(batch, lookahead=lookahead)  # metadata from pre-step state
        marks = []
        for seq in batch.seqs:
            seq.num_computed += 1
            marks.append((seq, len(seq.output_ids), seq.num_computed))
            seq.append(PENDING_TOKEN)  # filled in by _collect
        if lookahead:
            self.timing["lookahead_steps"] += 1
        return _Inflight(batch, h, marks, t0)

    def _lookahead_batch(self, cur: "_Inflight"):
        """The decode batch continuing ``cur`` row for row, or None to drain."""
        if not self.cfg.async_decode or self.scheduler.waiting:
            return None
        for seq, idx, _ in cur.marks:
            if seq.status != SeqStatus.RUNNING:
                return None
            if idx + 1 >= seq.sampling.max_tokens or \
                    seq.num_prompt + idx + 1 >= self.cfg.max_model_len:
                return None  # finishes by length at cur: nothing to look ahead for
        for seq in cur.batch.seqs:
            if not self.runner.bm.ensure(seq.seq_id, seq.num_tokens):
                return None  # KV pool full: the scheduler decides (preemption)
        n = len(cur.batch.seqs)
        return Batch(seqs=list(cur.batch.seqs), q_start=[s.num_computed for s in cur.batch.seqs],
                     q_len=[1] * n, num_decode=n)

    def _collect(self, cur: "_Inflight") -> list[RequestOutput]:
        toks = self.runner.collect(cur.handle)
        now = time.perf_counter()
        self.timing["execute"] += now - max(cur.t0, self._last_collect)
        self._last_collect = now
        self.timing["steps"] += 1
        outs = []
        for (seq, idx, ncomp), tok in zip(cur.marks, toks):
            if seq.status == SeqStatus.FINISHED:
                continue  # aborted while in flight
            tok = int(tok)
            seq.output_ids[idx] = tok
            seq._ids_np = None
            if seq.first_token_time is None:
                seq.first_token_time = now
            self.runner.bm.commit(seq.seq_id, seq.token_array(), ncomp)
            reason = self._stop_reason(seq, tok, idx + 1)
            if reason:
                del seq.output_ids[idx + 1:]  # drop a look-ahead placeholder
                seq._ids_np = None
                self.scheduler.finish(seq, reason)
            outs.append(self._output(seq, [tok], upto=idx + 1))
        self._account(cur.batch, len(outs), now - cur.t0)
        self.timing["post"] += time.perf_counter() - now
        return outs

    def _account(self, batch, n_out: int, seconds: float):
        self.total_steps += 1
        self.total_generated += n_out
        self.last_step = StepStats(len(batch.seqs), batch.num_tokens, batch.num_decode, seconds)
        self.batch_size_history.append(len(batch.seqs))
        if len(self.batch_size_history) > 4096:
            del self.batch_size_history[:2048]

    def _sync_step(self, batch, t0: float) -> list[RequestOutput]:
        with self.lock:
            toks = self.runner.execute(batch)
            now = time.perf_counter()
            self.timing["execute"] += now - t0
            self.timing["steps"] += 1
            outs = []
            for seq, n, tok in zip(batch.seqs, batch.q_len, toks):
                seq.num_computed += n
                if seq.num_computed < seq.num_tokens:
                    self.runner.bm.commit(seq.seq_id, seq.token_array(), seq.num_computed)
                    continue  # chunked prefill not finished: sampled token discarded
                tok = int(tok)
                seq.append(tok)
                if seq.first_token_time is None:
                    seq.first_token_time = now
                self.runner.bm.commit(seq.seq_id, seq.token_array(), seq.num_computed)
                reason = self._stop_reason(seq, tok)
                if reason:
                    self.scheduler.finish(seq, reason)
                outs.append(self._output(seq, [tok]))
            self._account(batch, len(outs), now - t0)
            self.timing["post"] += time.perf_counter() - now
            return outs

    def _stop_reason(self, seq: Sequence, tok: int, n_out: int | None = None) -> str | None:
        """``n_out``: output tokens up to and including ``tok`` (default: all of them)."""
        sp = seq.sampling
        n_out = len(seq.output_ids) if n_out is None else n_out
        if not sp.ignore_eos and (tok in self.eos_ids or tok in sp.stop_token_ids):
            return "stop"
        if n_out >= sp.max_tokens:
            return "length"
        if seq.num_prompt + n_out >= self.cfg.max_model_len:
            return "length"
        return None

    def _output(self, seq: Sequence, new, upto: int | None = None) -> RequestOutput:
        ids = seq.output_ids if upto is None else seq.output_ids[:upto]
        return RequestOutput(
            request_id=seq.request_id, token_ids=list(ids), finished=seq.finished,
            finish_reason=seq.finish_reason, prompt_tokens=seq.num_prompt,
            cached_prompt_tokens=seq.num_cached_prompt, arrival_time=seq.arrival_time,
            first_token_time=seq.first_token_time, first_scheduled_time=seq.first_scheduled_time,
            finish_time=seq.finish_time, new_token_ids=list(new))

    # ------------------------------------------------------------------------------------
    def generate(self, prompts, sampling: SamplingParams | list) -> list[RequestOutput]:
        """Blocking batch generation (prompts: list of token-id lists or strings)."""
        if not isinstance(sampling, list):
            sampling = [sampling] * len(prompts)
        ids = []
        for i, p in enumerate(prompts):
            toks = self.tokenizer.encode(p) if isinstance(p, str) else p
            rid = f"gen-{time.monotonic_ns()}-{i}"
            self.add_request(rid, toks, sampling[i])
            ids.append(rid)
        final: dict[str, RequestOutput] = {}
        while self.has_unfinished():
            for o in self.step():
                if o.finished:
                    final[o.request_id] = o
        return [final[r] for r in ids if r in final]

    # ------------------------------------------------------------------------------------
    def kv_cache_info(self) -> dict:
        r = self.runner
        return {
            "num_gpu_blocks": r.num_blocks,
            "block_size": r.block_size,
            "total_tokens": r.kv_total_tokens,
            "free_blocks": r.bm.num_free_blocks(),
            "cached_blocks": r.bm.num_cached_blocks(),
            "prefix_queries": r.bm.prefix_queries(),
            "prefix_hits": r.bm.prefix_hits(),
        }

    def shutdown(self):
        """Release engine resources (TP engines stop their worker ranks)."""

    def est_max_concurrency(self) -> float:
        return self.runner.kv_total_tokens / max(1, self.cfg.max_model_len)


def token_array(ids) -> np.ndarray:
    return np.asarray(ids, dtype=np.int64)
