"""Request / sequence state for the serving engine."""
from __future__ import annotations

import enum
import itertools
import time
from dataclasses import dataclass, field

import numpy as np


@dataclass
class SamplingParams:
    """Per-request sampling knobs.  The reference sends SamplingParams(temperature=0.2,
    max_tokens=...) to vLLM (llm/serve_llm.py:379, 520-525); top_p/top_k stay disabled by
    default like vLLM's defaults."""
    temperature: float = 0.2
    max_tokens: int = 512
    ignore_eos: bool = False
    seed: int | None = None
    stop_token_ids: tuple = ()
    top_p: float = 1.0
    top_k: int = -1


class SeqStatus(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2


_ids = itertools.count(1)


@dataclass
class Sequence:
    request_id: str
    prompt_ids: list
    sampling: SamplingParams
    arrival_time: float = field(default_factory=time.perf_counter)
    seq_id: int = field(default_factory=lambda: next(_ids))
    output_ids: list = field(default_factory=list)
    status: SeqStatus = SeqStatus.WAITING
    num_computed: int = 0          # tokens whose KV is in the cache
    num_cached_prompt: int = 0     # prompt tokens served by the prefix cache
    first_scheduled_time: float | None = None
    first_token_time: float | None = None
    finish_time: float | None = None
    finish_reason: str | None = None
    seed: int = 0
    num_preemptions: int = 0
    _ids_np: np.ndarray | None = None

    @property
    def num_prompt(self) -> int:
        return len(self.prompt_ids)

    @property
    def num_tokens(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids)

    @property
    def num_pending(self) -> int:
        """Tokens whose KV still has to be computed (1 = decode step)."""
        return self.num_tokens - self.num_computed

    @property
    def finished(self) -> bool:
        return self.status == SeqStatus.FINISHED

    def token_array(self) -> np.ndarray:
        """All token ids as int64 numpy (cached; extended lazily)."""
        n = self.num_tokens
        a = self._ids_np
        if a is None or a.shape[0] != n:
            a = np.asarray(self.prompt_ids + self.output_ids, dtype=np.int64)
            self._ids_np = a
        return a

    def append(self, tok: int):
        self.output_ids.append(int(tok))
        self._ids_np = None
