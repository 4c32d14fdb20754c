"""Randomised stress of the continuous-batching scheduler over the native C++ block manager
(SURVEY §5.2 "stress tests of the scheduler"): bursty arrivals, a KV pool small enough to
force preemption, shared prefixes (prefix-cache hits), random aborts and chunked prefill.
No model runs - the test drives Scheduler + BlockManager directly and checks the invariants
every step:

* the step's tokens fit max_num_batched_tokens, running sequences fit max_num_seqs;
* decodes come first and carry exactly one token; prefill chunks start at num_computed;
* every scheduled sequence owns enough KV blocks for the tokens it computes;
* no KV block is owned twice unless prefix caching shares it;
* at the end every request finished with exactly max_tokens outputs (or was aborted) and
  the pool is whole again.
"""
import random

import numpy as np
import pytest

from agentic_traffic_testing_amd.engine.scheduler import Scheduler
from agentic_traffic_testing_amd.engine.sequence import SamplingParams, Sequence, SeqStatus
from agentic_traffic_testing_amd.runtime import BlockManager


def _run(seed: int, num_blocks: int, block_size: int, max_seqs: int, budget: int,
         prefix_caching: bool, long_prefill: int):
    rng = random.Random(seed)
    max_model_len = 512
    bm = BlockManager(num_blocks, block_size, prefix_caching)
    sch = Scheduler(bm, max_seqs, budget, max_model_len, long_prefill)
    shared = [rng.randrange(300, 3000) for _ in range(3 * block_size)]
    live: dict[str, Sequence] = {}
    done: dict[str, Sequence] = {}
    aborted: set[str] = set()
    n_req = 0
    for _ in range(4000):
        # bursty arrivals: nothing for a while, then a fan-out of up to 6 requests
        if n_req < 60 and rng.random() < 0.08:
            for _ in range(rng.randint(1, 6)):
                plen = rng.randint(1, 160)
                prompt = shared[:rng.randint(0, len(shared))] if rng.random() < 0.5 else []
                prompt = (prompt + [rng.randrange(300, 3000) for _ in range(plen)])[:300]
                s = Sequence(f"r{n_req}", prompt,
                             SamplingParams(max_tokens=rng.randint(1, 40), ignore_eos=True))
                n_req += 1
                live[s.request_id] = s
                sch.add(s)
        if live and rng.random() < 0.01:
            rid = rng.choice(sorted(live))
            for s in sch.abort(rid):
                aborted.add(s.request_id)
                live.pop(s.request_id, None)
        b = sch.schedule()
        assert len(sch.running) <= max_seqs
        assert b.num_tokens <= budget
        assert all(q == 1 for q in b.q_len[:b.num_decode])
        owned: dict[int, int] = {}
        for s, qs, ql in zip(b.seqs, b.q_start, b.q_len):
            assert s.status == SeqStatus.RUNNING and qs == s.num_computed and ql >= 1
            assert qs + ql <= s.num_tokens
            blocks = bm.blocks(s.seq_id)
            assert len(blocks) * block_size >= qs + ql, (len(blocks), qs, ql)
            assert len(set(blocks)) == len(blocks)
            for blk in blocks:
                assert 0 <= blk < num_blocks
                if blk in owned and not prefix_caching:
                    pytest.fail(f"block {blk} owned twice without prefix caching")
                owned[blk] = owned.get(blk, 0) + 1
        # "execute": the scheduled tokens' KV is now computed; a sequence whose pending
        # tokens are all computed emits one token
        for s, ql in zip(b.seqs, b.q_len):
            s.num_computed += ql
            bm.commit(s.seq_id, s.token_array(), s.num_computed)
            if s.num_computed == s.num_tokens:
                s.append(rng.randrange(300, 3000))
                if len(s.output_ids) >= s.sampling.max_tokens:
                    sch.finish(s, "length")
                    done[s.request_id] = live.pop(s.request_id)
        if n_req >= 60 and not sch.has_work():
            break
    assert not sch.has_work(), "scheduler did not drain"
    assert set(done) | aborted == {f"r{i}" for i in range(n_req)}
    for s in done.values():
        assert len(s.output_ids) == s.sampling.max_tokens
    assert bm.num_free_blocks() == num_blocks
    return sch


@pytest.mark.parametrize("seed", range(6))
def test_scheduler_stress(seed):
    _run(seed, num_blocks=48, block_size=16, max_seqs=8, budget=96,
         prefix_caching=seed % 2 == 0, long_prefill=64 if seed % 3 == 0 else 0)


def test_scheduler_stress_forces_preemption():
    sch = _run(11, num_blocks=20, block_size=16, max_seqs=12, budget=256,
               prefix_caching=False, long_prefill=0)
    assert sch.num_preemptions > 0


def test_block_manager_prefix_sharing_refcounts():
    bm = BlockManager(8, 4, True)
    toks = np.arange(100, 113, dtype=np.int64)  # 3 full blocks + 1 token
    assert bm.allocate(1, toks, 14) == 0
    bm.commit(1, toks, 13)
    # same prefix: the three full blocks are served from the cache and shared
    assert bm.allocate(2, toks, 14) == 12
    shared = set(bm.blocks(1)[:3])
    assert shared == set(bm.blocks(2)[:3])
    bm.free(1)
    assert set(bm.blocks(2)[:3]) == shared  # still owned by seq 2
    bm.free(2)
    assert bm.num_free_blocks() == 8
