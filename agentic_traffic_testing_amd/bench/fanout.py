"""5-agent fan-out workload (BASELINE.md "Measurement protocol").

One *episode* replays the LLM arrival shape of Agent A's ``agentic_parallel`` scenario
(reference agents/agent_a/server.py:441-648):

  1 planning request  ->  N (=5) concurrent Agent-B requests  ->  1 final synthesis request

Prompts are built exactly like the reference builds them (planner prompt, the
"You are Agent B.\\n<role/contract>\\n\\n<subtask>" worker prompt with the
``_parse_subtasks`` fallback subtasks that random-init weights always produce, and the
critic prompt embedding every worker report), wrapped in the Llama-3 chat template and
truncated like llm/serve_llm.py:810-844.  Generation is fixed to ``max_tokens``
(ignore_eos) so every episode does identical work.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np

from ..engine.sequence import SamplingParams
from ..engine.tokenizer import apply_chat_template

TASKS = [
    "A school is designing a small amusement park with three rides. The first ride costs "
    "$500 to build and makes $20 per ride. The second ride costs $700 and makes $25 per ride. "
    "The third ride costs $900 and makes $30 per ride. The school has a budget of $2000 and "
    "wants to maximize revenue in 1 day if 100 students ride each ride at most once. "
    "Determine which rides to build and calculate the expected total revenue.",
    "Research the current state of quantum computing and its potential applications in "
    "cryptography. Provide a comprehensive summary with key findings and recommendations.",
    "Design and implement a Python calculator with a graphical user interface that supports "
    "basic arithmetic operations, keyboard input, and error handling.",
    "Provide recommendations for a startup looking to implement AI-powered customer service. "
    "Consider cost, scalability, user experience, and implementation timeline.",
]

AGENT_B_ROLES = ["researcher", "analyst", "engineer", "critic", "summarizer"]


def planning_prompt(task: str, n: int) -> str:
    return ("You are Agent A, acting as the planner. Break the user task into "
            f"{n} concrete, independent subtasks. Return ONLY valid JSON "
            'as an array of strings, e.g. ["subtask 1", "subtask 2"].\n\n'
            f"User task:\n{task}")


def worker_prompt(subtask: str, role: str) -> str:
    return f"You are Agent B.\nRole: {role}\n\n{subtask}"


def final_prompt(task: str, reports: list[str]) -> str:
    lines = [f"Worker {i} (http://agent-b-{i}:{8101 + i}/subtask):\nSubtask: Subtask {i}: {task}\n{r}"
             for i, r in enumerate(reports, start=1)]
    return ("You are Agent A acting as planner/critic. Review the worker reports, "
            "note inconsistencies or gaps, then produce the best final response to the user.\n\n"
            f"User task:\n{task}\n\nWorker reports:\n" + "\n\n".join(lines))


@dataclass
class EpisodeResult:
    completion_tokens: int = 0
    prompt_tokens: int = 0
    cached_prompt_tokens: int = 0
    ttfts: list = field(default_factory=list)
    latencies: list = field(default_factory=list)
    seconds: float = 0.0
    requests: int = 0
    # per phase (planning / burst / final): (name, prompt tokens, cached tokens, TTFTs)
    phases: list = field(default_factory=list)


class FanoutWorkload:
    def __init__(self, engine, fanout: int = 5, max_tokens: int = 512, temperature: float = 0.2,
                 safety_margin: int = 128, seed: int = 0):
        self.engine = engine
        self.tok = engine.tokenizer
        self.fanout = fanout
        self.max_tokens = max_tokens
        self.temperature = temperature
        self.margin = safety_margin
        self.rng = np.random.default_rng(seed)
        self.episode_idx = 0

    def _encode(self, text: str) -> list[int]:
        ids = self.tok.encode(apply_chat_template(text))
        limit = max(0, self.engine.cfg.max_model_len - self.max_tokens - self.margin)
        return ids[:limit] if len(ids) > limit else ids

    def _sp(self) -> SamplingParams:
        return SamplingParams(temperature=self.temperature, max_tokens=self.max_tokens,
                              ignore_eos=True, seed=int(self.rng.integers(1 << 62)))

    def _run_phase(self, prompts: list[list[int]], res: EpisodeResult, name: str = "") -> list:
        eng = self.engine
        t_arr = time.perf_counter()
        rids = []
        for i, p in enumerate(prompts):
            rid = f"ep{self.episode_idx}-{len(res.latencies) + i}"
            eng.add_request(rid, p, self._sp(), arrival_time=t_arr)
            rids.append(rid)
        done = {}
        while len(done) < len(rids):
            for o in eng.step():
                if o.finished:
                    done[o.request_id] = o
        outs = [done[r] for r in rids]
        for o in outs:
            res.completion_tokens += o.completion_tokens
            res.prompt_tokens += o.prompt_tokens
            res.cached_prompt_tokens += o.cached_prompt_tokens
            res.ttfts.append(o.ttft)
            res.latencies.append(o.finish_time - o.arrival_time)
            res.requests += 1
        res.phases.append((name, sum(o.prompt_tokens for o in outs),
                           sum(o.cached_prompt_tokens for o in outs), [o.ttft for o in outs]))
        return outs

    def run_episode(self) -> EpisodeResult:
        task = TASKS[self.episode_idx % len(TASKS)] + f" (episode {self.episode_idx})"
        res = EpisodeResult()
        t0 = time.perf_counter()
        self._run_phase([self._encode(planning_prompt(task, self.fanout))], res, "planning")
        subtasks = [f"Subtask {i}: {task}" for i in range(1, self.fanout + 1)]
        worker_ids = [self._encode(worker_prompt(s, AGENT_B_ROLES[i % len(AGENT_B_ROLES)]))
                      for i, s in enumerate(subtasks)]
        outs = self._run_phase(worker_ids, res, "burst")
        reports = [self.tok.decode(o.token_ids) for o in outs]
        self._run_phase([self._encode(final_prompt(task, reports))], res, "final")
        res.seconds = time.perf_counter() - t0
        self.episode_idx += 1
        return res
