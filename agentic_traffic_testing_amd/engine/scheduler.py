"""Continuous-batching scheduler tuned for agent fan-out bursts.

Replaces vLLM's scheduler that the reference configures through ``max_num_seqs`` and
``max_num_batched_tokens`` (llm/serve_llm.py:362-373; compose defaults 12 / 8192).

Policy per step (token budget = max_num_batched_tokens):

1. **Decodes first** (stall-free batching): every running sequence with one pending token
   gets it, so a burst of new prompts never freezes in-flight generations.  If the KV pool
   cannot grow a sequence, the most recently admitted sequence is preempted (its blocks
   are freed; it is recomputed later - prefix caching usually makes that cheap).
2. **Ongoing chunked prefills** continue with whatever budget is left.
3. **Admission**: waiting requests are admitted FIFO while ``max_num_seqs`` and the budget
   allow.  An agent-a -> N x agent-b fan-out arrives within milliseconds;
   admitting all N in the same step batches their prefills into one forward, and their
   shared templated prefix is served from the prefix cache after the first one.

The output is a ``Batch`` whose sequences are ordered decode-first, matching the
attention kernels' split (decode kernel over [0, num_decode), prefill tiles after).
"""
from __future__ import annotations

import collections
import time
from dataclasses import dataclass, field

import numpy as np

from .sequence import Sequence, SeqStatus


@dataclass
class Batch:
    seqs: list = field(default_factory=list)
    q_start: list = field(default_factory=list)
    q_len: list = field(default_factory=list)
    num_decode: int = 0
    preempted: list = field(default_factory=list)

    @property
    def num_tokens(self) -> int:
        return int(sum(self.q_len))

    @property
    def empty(self) -> bool:
        return not self.seqs

    def arrays(self):
        return (np.fromiter((s.seq_id for s in self.seqs), dtype=np.int64, count=len(self.seqs)),
                np.asarray(self.q_start, dtype=np.int64), np.asarray(self.q_len, dtype=np.int64))


class Scheduler:
    def __init__(self, block_manager, max_num_seqs: int, max_num_batched_tokens: int,
                 max_model_len: int, long_prefill_token_threshold: int = 0):
        self.bm = block_manager
        self.max_num_seqs = max_num_seqs
        self.max_num_batched_tokens = max_num_batched_tokens
        self.max_model_len = max_model_len
        self.long_prefill = long_prefill_token_threshold or max_num_batched_tokens
        self.waiting: collections.deque[Sequence] = collections.deque()
        self.running: list[Sequence] = []
        self.num_preemptions = 0

    # ------------------------------------------------------------------------------------
    def add(self, seq: Sequence):
        seq.status = SeqStatus.WAITING
        self.waiting.append(seq)

    def abort(self, request_id: str) -> list[Sequence]:
        out = []
        for s in list(self.waiting):
            if s.request_id == request_id:
                self.waiting.remove(s)
                out.append(s)
        for s in list(self.running):
            if s.request_id == request_id:
                self.running.remove(s)
                self.bm.free(s.seq_id)
                out.append(s)
        for s in out:
            s.status = SeqStatus.FINISHED
            s.finish_reason = "abort"
        return out

    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    def num_waiting(self) -> int:
        return len(self.waiting)

    # ------------------------------------------------------------------------------------
    def _preempt(self, seq: Sequence):
        self.bm.free(seq.seq_id)
        seq.num_computed = 0
        seq.status = SeqStatus.WAITING
        seq.num_preemptions += 1
        self.num_preemptions += 1
        self.waiting.appendleft(seq)

    def schedule(self) -> Batch:
        budget = self.max_num_batched_tokens
        decodes: list[Sequence] = []
        prefills: list[tuple[Sequence, int]] = []
        b = Batch()

        # 1. decodes (one pending token)
        for seq in list(self.running):
            if seq not in self.running or seq.num_pending != 1:
                continue
            while not self.bm.ensure(seq.seq_id, seq.num_tokens):
                victim = self.running[-1]
                self.running.remove(victim)
                self._preempt(victim)
                b.preempted.append(victim)
                if victim is seq:
                    break
            if seq.status != SeqStatus.RUNNING:
                continue
            if budget <= 0:
                break
            decodes.append(seq)
            budget -= 1
        if b.preempted:  # a victim may have been picked after it was scheduled
            kept = [s for s in decodes if s.status == SeqStatus.RUNNING]
            budget += len(decodes) - len(kept)
            decodes = kept

        # 2. ongoing chunked prefills
        for seq in self.running:
            if seq.num_pending <= 1 or budget <= 0:
                continue
            n = min(seq.num_pending, budget, self.long_prefill)
            prefills.append((seq, n))
            budget -= n

        # 3. admission
        while self.waiting and budget > 0 and len(self.running) < self.max_num_seqs:
            seq = self.waiting[0]
            reserve = min(seq.num_tokens + 1, self.max_model_len)
            cached = self.bm.allocate(seq.seq_id, seq.token_array(), reserve)
            if cached < 0:
                break  # KV pool full: wait for running sequences to finish
            self.waiting.popleft()
            seq.num_computed = int(cached)
            if seq.num_preemptions == 0:
                seq.num_cached_prompt = int(cached)
            seq.status = SeqStatus.RUNNING
            if seq.first_scheduled_time is None:
                seq.first_scheduled_time = time.perf_counter()
            self.running.append(seq)
            n = min(seq.num_pending, budget, self.long_prefill)
            if n == 1:
                decodes.append(seq)
            else:
                prefills.append((seq, n))
            budget -= n

        for seq in decodes:
            b.seqs.append(seq)
            b.q_start.append(seq.num_computed)
            b.q_len.append(1)
        b.num_decode = len(decodes)
        for seq, n in prefills:
            b.seqs.append(seq)
            b.q_start.append(seq.num_computed)
            b.q_len.append(n)
        return b

    # ------------------------------------------------------------------------------------
    def finish(self, seq: Sequence, reason: str):
        seq.status = SeqStatus.FINISHED
        seq.finish_reason = reason
        seq.finish_time = time.perf_counter()
        if seq in self.running:
            self.running.remove(seq)
        self.bm.free(seq.seq_id)
