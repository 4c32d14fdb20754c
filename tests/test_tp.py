"""Tensor parallelism on CPU (gloo, world_size 2): comm primitives, the shared-memory
step channel and a full TP=2 engine against TP=1."""
import multiprocessing as mp
import os

import numpy as np
import pytest
import torch

from agentic_traffic_testing_amd import ops
from agentic_traffic_testing_amd.config import EngineConfig
from agentic_traffic_testing_amd.engine.llm_engine import LLMEngine
from agentic_traffic_testing_amd.engine.sequence import SamplingParams
from agentic_traffic_testing_amd.ops import reference as ref
from agentic_traffic_testing_amd.parallel.tp_engine import TPEngine, free_port
from agentic_traffic_testing_amd.runtime import ShmChannel


def test_shm_channel_roundtrip():
    w = ShmChannel("atta_pytest_chan", 64, 2, create=True)
    r = ShmChannel("atta_pytest_chan")
    assert w.publish(np.arange(5, dtype=np.int32)) == 1
    for reader in (0, 1):
        seq, data = r.receive(reader, 0, 1.0)
        assert seq == 1 and data.tolist() == [0, 1, 2, 3, 4]
    assert w.publish(np.array([7], dtype=np.int32)) == 2
    assert r.receive(1, 1, 1.0)[1].tolist() == [7]
    # reader 0 has not acked message 2 yet: a third publish must wait, and time out
    with pytest.raises(RuntimeError):
        w.publish(np.array([8], dtype=np.int32), 0.05)
    assert r.receive(0, 1, 1.0)[1].tolist() == [7]
    assert r.receive(0, 2, 0.01) is None  # nothing new
    with pytest.raises(Exception):
        w.publish(np.zeros(65, dtype=np.int32))  # over capacity
    w.close()
    assert r.receive(0, 2, -1) is None  # closed channel wakes blocked readers


def _register_and_exit(name, reader):
    ShmChannel(name).register_reader(reader)


def _create_and_exit(name, q):
    ch = ShmChannel(name, 16, 1, create=True)  # noqa: F841  (the segment outlives no one)
    q.put("created")
    import time

    time.sleep(0.5)
    os._exit(0)  # skip the destructor's shm_unlink: the segment stays, its writer is gone


def test_shm_channel_rank_liveness():
    """SURVEY §5.3 TP-rank liveness: rank 0 names a dead worker instead of waiting forever,
    and a worker can tell that rank 0 is gone."""
    name = f"atta_pytest_live_{os.getpid()}"
    w = ShmChannel(name, 16, 2, create=True)
    assert w.writer_alive and w.dead_readers() == []
    w.register_reader(0)  # reader 0 = this (live) process
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_register_and_exit, args=(name, 1))
    p.start()
    p.join(60)
    assert w.dead_readers() == [1]
    w.publish(np.zeros(1, dtype=np.int32))  # seq 1: nobody has to have acked seq 0
    ShmChannel(name).receive(0, 0, 1.0)
    with pytest.raises(RuntimeError, match="died"):
        w.publish(np.zeros(1, dtype=np.int32), 30.0)  # reader 1 never acks, and is dead
    del w

    name2 = name + "_w"
    q = ctx.Queue()
    p = ctx.Process(target=_create_and_exit, args=(name2, q))
    p.start()
    assert q.get(timeout=60) == "created"
    r = ShmChannel(name2)
    p.join(60)
    assert not r.writer_alive
    assert r.receive(0, 0, 0.05) is None
    os.remove(f"/dev/shm/{name2}")


def _comm_worker(rank, world, port, q):
    try:
        from agentic_traffic_testing_amd.parallel.comm import init_distributed

        comm = init_distributed(rank, world, "cpu", "gloo", "127.0.0.1", port)
        x = torch.full((3, 4), float(rank + 1), dtype=torch.bfloat16)
        comm.all_reduce(x)
        g = comm.all_gather_last(torch.full((2, 3), float(rank)))
        # vocab-parallel sampling: MAX of the per-shard keys == sampling the full logits
        torch.manual_seed(0)
        logits = torch.randn(4, 64)
        temp = torch.tensor([0.0, 0.7, 1.0, 0.2])
        seeds = torch.tensor([1, 2, 3, 4])
        steps = torch.tensor([0, 5, 9, 100])
        shard = logits[:, rank * 32:(rank + 1) * 32]
        keys = ref.sample_keys(shard, temp, seeds, steps, vocab_offset=rank * 32)
        comm.all_reduce_max(keys)
        from agentic_traffic_testing_amd.ops import key_to_token

        toks = key_to_token(keys)
        full = ref.sample(logits, temp, seeds, steps)
        q.put((rank, float(x.float().mean()), g.tolist(), toks.tolist(), full.tolist(),
               comm.min_int(10 + rank, "cpu")))
        torch.distributed.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, repr(e)))


def test_comm_primitives_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_comm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r in res:
        assert len(r) == 6, r
        rank, mean, g, toks, full, mn = r
        assert mean == 3.0
        assert g == [[0.0, 0.0, 0.0, 1.0, 1.0, 1.0]] * 2
        assert toks == full
        assert mn == 10


def _prompts():
    rng = np.random.default_rng(7)
    return [rng.integers(300, 3000, size=n).tolist() for n in (33, 9, 70)]


@pytest.mark.parametrize("tp,model", [(2, "tiny"), (4, "tiny-tp8"), (8, "tiny-tp8")])
def test_tp_engine_matches_tp1_cpu(tp, model):
    """TP=2/4/8 against TP=1.  tiny-tp8 has 8 q heads over 2 KV heads, so TP=4 and TP=8
    replicate every KV head over 2 / 4 ranks (kv_rep > 1, models/llama.py)."""
    base = dict(model=model, device="cpu", dtype="float32", max_model_len=256,
                num_kv_blocks=64, max_num_batched_tokens=64, max_num_seqs=4, use_graphs=False)
    greedy = SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True)
    sampled = SamplingParams(temperature=0.8, max_tokens=8, ignore_eos=True, seed=11)
    ref_eng = LLMEngine(EngineConfig(**base))
    n_heads, n_kv, inter = (ref_eng.runner.model.n_heads, ref_eng.runner.model.n_kv_heads,
                            ref_eng.runner.model.inter)
    exp_g = [o.token_ids for o in ref_eng.generate(_prompts(), greedy)]
    exp_s = [o.token_ids for o in ref_eng.generate(_prompts(), sampled)]
    topp = SamplingParams(temperature=0.7, top_p=0.9, top_k=40, max_tokens=4, ignore_eos=True,
                          seed=3)
    exp_p = [o.token_ids for o in ref_eng.generate(_prompts()[:2], topp)]
    del ref_eng
    eng = TPEngine(EngineConfig(tensor_parallel_size=tp, **base))
    try:
        m = eng.runner.model
        assert m.n_heads == n_heads // tp and m.inter == inter // tp
        assert m.kv_rep == max(1, tp // n_kv) and m.n_kv_heads == max(1, n_kv // tp)
        got_g = [o.token_ids for o in eng.generate(_prompts(), greedy)]
        got_s = [o.token_ids for o in eng.generate(_prompts(), sampled)]
        # top-k / top-p: every rank samples the all-gathered logits with the same kernel
        got_p = [o.token_ids for o in eng.generate(_prompts()[:2], topp)]
    finally:
        eng.shutdown()
    assert got_g == exp_g
    assert got_s == exp_s
    assert got_p == exp_p
    assert not any(p.is_alive() for p in eng.procs)


@pytest.mark.parametrize("tp,model", [(2, "tiny"), (4, "tiny-tp8")])
def test_tp_fp8_engine_matches_tp1_fp8_cpu(tp, model):
    """VERDICT r4 #4 (BASELINE config 5 = TP x fp8): TP=2/4 with fp8 weight-only quantisation
    against TP=1 fp8 on the dequantised CPU reference path.  Row-parallel shards (o, down)
    quantise with the full row's scale (models/llama.py _make_layer), so every rank holds the
    TP=1 fp8 values exactly and only the partial-sum order differs (fp32 here)."""
    base = dict(model=model, device="cpu", dtype="float32", max_model_len=256,
                num_kv_blocks=64, max_num_batched_tokens=64, max_num_seqs=4, use_graphs=False,
                quantization="fp8")
    greedy = SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True)
    sampled = SamplingParams(temperature=0.8, max_tokens=8, ignore_eos=True, seed=13)
    ref_eng = LLMEngine(EngineConfig(**base))
    m1 = ref_eng.runner.model
    o_full = torch.cat([L.o for L in m1.layers[:1]], 0).clone()
    exp_g = [o.token_ids for o in ref_eng.generate(_prompts(), greedy)]
    exp_s = [o.token_ids for o in ref_eng.generate(_prompts(), sampled)]
    # the fp8 weights are really fp8-valued: re-quantising them changes nothing
    from agentic_traffic_testing_amd import ops
    q, sc = ops.quantize_fp8(o_full)
    assert torch.equal(ops.dequantize_fp8(q, sc, o_full.dtype), o_full)
    del ref_eng
    eng = TPEngine(EngineConfig(tensor_parallel_size=tp, **base))
    try:
        assert eng.runner.model.quant == "fp8"
        got_g = [o.token_ids for o in eng.generate(_prompts(), greedy)]
        got_s = [o.token_ids for o in eng.generate(_prompts(), sampled)]
    finally:
        eng.shutdown()
    assert got_g == exp_g
    assert got_s == exp_s


def test_fp8_row_parallel_shards_use_full_row_scale():
    """The o / down shards of every TP rank dequantise to the TP=1 fp8 weights' K slice."""
    from agentic_traffic_testing_amd.config import resolve_model
    from agentic_traffic_testing_amd.models.llama import LlamaModel

    mcfg = resolve_model("tiny")[0]
    full = LlamaModel(mcfg, torch.float32, "cpu", quantization="fp8").init_random(seed=5)
    for tp in (2, 4):
        for r in range(tp):
            m = LlamaModel(mcfg, torch.float32, "cpu", tp_rank=r, tp_size=tp,
                           quantization="fp8").init_random(seed=5)
            for L, F in zip(m.layers, full.layers):
                k_o, k_d = L.o.shape[1], L.down.shape[1]
                assert torch.equal(L.o, F.o[:, r * k_o:(r + 1) * k_o])
                assert torch.equal(L.down, F.down[:, r * k_d:(r + 1) * k_d])


def test_tp_step_failure_stops_the_group():
    """a step that raises after rank 0 published it must stop the whole TP group
    (workers exit, the serving loop dies -> /health 503) instead of continuing with ranks
    whose collectives no longer pair up."""
    import asyncio
    import time

    from agentic_traffic_testing_amd.engine.async_engine import AsyncEngine

    base = dict(model="tiny", device="cpu", dtype="float32", max_model_len=256,
                num_kv_blocks=64, max_num_batched_tokens=64, max_num_seqs=4, use_graphs=False)
    eng = TPEngine(EngineConfig(tensor_parallel_size=2, **base))
    runner = eng.runner
    orig = runner._run

    def failing_run(hdr, sampler=None, worker=False):
        raise RuntimeError("injected failure after publish")

    runner._run = failing_run
    ae = AsyncEngine(eng).start()
    try:
        async def go():
            sp = SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True)
            with pytest.raises(RuntimeError):
                async for _ in ae.generate([300, 301, 302], sp, "r0"):
                    pass

        asyncio.run(go())
        t0 = time.monotonic()
        while ae.alive and time.monotonic() - t0 < 30:
            time.sleep(0.05)
        assert not ae.alive, "engine loop kept running after a failed TP step"
        assert "TP step failed" in (ae.last_error or "")
        for p in eng.procs:
            p.join(30)
        assert not any(p.is_alive() for p in eng.procs)
    finally:
        runner._run = orig
        ae._stop.set()
        eng.kill()


def test_shm_channel_registration_deadline():
    """a reader that never registers (died while loading weights) is reported
    dead once the registration deadline passes, so rank 0's publish fails instead of
    blocking forever."""
    import time

    name = f"atta_pytest_reg_{os.getpid()}"
    w = ShmChannel(name, 16, 1, create=True, register_timeout_s=0.3)
    assert w.unregistered_readers() == [0] and w.dead_readers() == []
    w.publish(np.zeros(1, dtype=np.int32))  # seq 1: nothing to wait for yet
    time.sleep(0.4)
    assert w.dead_readers() == [0]
    with pytest.raises(RuntimeError, match="died"):
        w.publish(np.zeros(1, dtype=np.int32), 30.0)
    del w
    # no deadline (0): an unregistered reader is only slow, never dead
    w = ShmChannel(name, 16, 1, create=True)
    w.publish(np.zeros(1, dtype=np.int32))
    with pytest.raises(RuntimeError, match="in time"):
        w.publish(np.zeros(1, dtype=np.int32), 0.2)


def _check_tp_greedy(m1, got, exp):
    """TP greedy tokens vs TP=1: the first token equal for all but one sequence, and every TP
    position teacher-forced against the fp32 dense oracle of the same weights:
    a mismatch must be a near tie (< 0.25 logit) and at most one position in five may differ -
    random-init weights make near-tie flips common (a row-parallel rank sums its K slice in a
    different order), so whole-sequence equality with TP=1 is not required."""
    from helpers import dense_logits
    assert sum(g[0] == e[0] for g, e in zip(got, exp)) >= len(got) - 1, (got, exp)
    bad_pos = checked = 0
    for p_, g in zip(_prompts(), got):
        ids = list(p_)
        for t in g:
            lg = dense_logits(m1, ids)
            checked += 1
            if int(torch.argmax(lg)) != t:
                assert float(lg.max() - lg[t]) < 0.25, (g, len(ids) - len(p_))
                bad_pos += 1
            ids.append(t)
    assert bad_pos <= checked // 5, (bad_pos, checked, got, exp)


@pytest.mark.gpu
def test_tp2_same_gpu_rehearsal_host_collectives():
    """Two TP ranks on ONE MI355X with the host-staged gloo collectives (RCCL refuses
    duplicate devices; tp_allreduce=auto installs no IPC there): eager steps, the fused decode
    path's vocab-parallel sampler and the step-channel protocol on real kernels."""
    base = dict(model="small", device="cuda:0", max_model_len=512, num_kv_blocks=256,
                max_num_batched_tokens=256, max_num_seqs=4, use_graphs=False)
    greedy = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True)
    ref_eng = LLMEngine(EngineConfig(**base))
    exp = [o.token_ids for o in ref_eng.generate(_prompts(), greedy)]
    m1 = ref_eng.runner.model  # the same seeded weights the TP ranks shard
    del ref_eng
    torch.cuda.empty_cache()
    eng = TPEngine(EngineConfig(tensor_parallel_size=2, tp_same_device=True, **base))
    try:
        got = [o.token_ids for o in eng.generate(_prompts(), greedy)]
        topp = SamplingParams(temperature=0.7, top_p=0.9, top_k=40, max_tokens=4,
                              ignore_eos=True, seed=5)
        assert all(len(o.token_ids) == 4 for o in eng.generate(_prompts()[:2], topp))
        assert eng.comm.ipc is None and eng.runner.graph_steps == 0
    finally:
        eng.shutdown()
    # bf16 partial sums split across ranks round differently: allow a late near-tie flip
    _check_tp_greedy(m1, got, exp)


@pytest.mark.gpu
@pytest.mark.parametrize("tp,model,push", [(2, "small", True), (4, "llama-70b-tp-slice", True),
                                           (8, "llama-70b-tp-slice", True),
                                           (8, "llama-70b-tp-slice", False)])
def test_tp_same_gpu_graph_captured_decode(tp, model, push):
    """TP=2/4/8 on ONE MI355X with hipGraph-captured decode.  Every decode-step
    collective is an IPC kernel on the peer buffers (X1/X2 sums with the residual add fused
    into the epilogue, X4 sampler-key MAX writing the token ids), so the whole step - every
    rank's 5 kernels x layers + 2 all-reduces per layer + LM head + key MAX - is captured and
    replayed although the control group is gloo.  Greedy tokens: _check_tp_greedy; the IPC
    timeout word stays 0.  push=True (the default): the o / down GEMVs push their partials
    straight into the peers' slots (fused push) and one receive kernel per projection adds the
    sum into the residual; push=False: GEMV + one-shot kernel."""
    base = dict(model=model, device="cuda:0", max_model_len=512, num_kv_blocks=128,
                max_num_batched_tokens=256, max_num_seqs=4, use_graphs=True)
    greedy = SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True)
    ref_eng = LLMEngine(EngineConfig(**base))
    exp = [o.token_ids for o in ref_eng.generate(_prompts(), greedy)]
    assert ref_eng.runner.graph_steps > 0
    m1 = ref_eng.runner.model  # the same seeded weights the TP ranks shard
    del ref_eng
    torch.cuda.empty_cache()
    eng = TPEngine(EngineConfig(tensor_parallel_size=tp, tp_same_device=True,
                                tp_allreduce="ipc", tp_fused_push=push, **base))
    try:
        r = eng.runner
        assert eng.comm.decode_capturable and r.graphs, "no decode graph was captured"
        steps0 = r.graph_steps
        got = [o.token_ids for o in eng.generate(_prompts(), greedy)]
        assert r.graph_steps > steps0, "TP decode steps did not replay from graphs"
        sampled = SamplingParams(temperature=0.8, max_tokens=6, ignore_eos=True, seed=9)
        s1 = [o.token_ids for o in eng.generate(_prompts(), sampled)]
        s2 = [o.token_ids for o in eng.generate(_prompts(), sampled)]
        assert s1 == s2  # seeded Gumbel draws: replay-deterministic across the TP group
        ipc = eng.comm.ipc
        assert ipc.calls_max > 0
        assert (ipc.calls_push > 0) if push else (ipc.calls > 0 and ipc.calls_push == 0)
        assert ipc.check() == 0
    finally:
        eng.shutdown()
    _check_tp_greedy(m1, got, exp)


@pytest.mark.gpu
@pytest.mark.parametrize("tp", [4, 8])
def test_tp_fp8_same_gpu_graph_captured_decode(tp):
    """BASELINE config 5 (TP x fp8) as a same-GPU rehearsal on the 70B TP=8
    per-rank geometry slice (FFN shard a multiple of the fp8 GEMV's 256-wide K step): fp8
    weight-only GEMVs on every rank, the all-reduce push fused into the o / down fp8 GEMV
    epilogues, graph-captured decode.  Same fp8 weights as TP=1 bit for bit (row-parallel
    shards quantise with the full-row scale); >= 95 % of decode steps replay from graphs, IPC
    word stays 0.

    Prefill rows quantise their activations per token (fp8 GEMMs); a row-parallel rank (o,
    down) scales its own K slice, so TP prefill numerics differ from TP=1 by that rounding.
    Every generated position is therefore checked teacher-forced against the fp32 oracle of
    the TP=1 fp8 weights (tests/helpers.py dense_logits_fp8, near-tie rule < 0.3 logits, at
    most one divergent position in five), not token-for-token against TP=1."""
    from helpers import dense_logits_fp8

    base = dict(model="llama-70b-tp-slice-fp8", device="cuda:0", max_model_len=512,
                num_kv_blocks=128, max_num_batched_tokens=256, max_num_seqs=4,
                use_graphs=True, quantization="fp8")
    greedy = SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True)
    ref_eng = LLMEngine(EngineConfig(**base))
    exp = [o.token_ids for o in ref_eng.generate(_prompts(), greedy)]
    assert ref_eng.runner.graph_steps > 0
    m1 = ref_eng.runner.model
    eng = TPEngine(EngineConfig(tensor_parallel_size=tp, tp_same_device=True,
                                tp_allreduce="ipc", tp_fused_push=True, **base))
    try:
        r = eng.runner
        assert r.model.quant == "fp8" and r.model.layers[0].o_s is not None
        assert eng.comm.decode_capturable and r.graphs, "no decode graph was captured"
        steps0, g0 = r.steps, r.graph_steps
        got = [o.token_ids for o in eng.generate(_prompts(), greedy)]
        decode_steps = r.steps - steps0 - 1  # one prefill step (all prompts fit one batch)
        assert r.graph_steps - g0 >= 0.95 * decode_steps, (r.graph_steps - g0, decode_steps)
        ipc = eng.comm.ipc
        assert ipc.calls_push > 0 and ipc.check() == 0
        eng_fused = r.model.small_prefill_ok(sum(len(p) for p in _prompts()))
    finally:
        eng.shutdown()
    # teacher-forced against the oracle (random-init weights make near ties common, and one
    # flip changes every later token of a sequence, so sequence equality with TP=1 is not
    # required).  The 112-row prefill runs the fused weight-only kernels (wide W8 builds:
    # 16-bit activations, like decode); a library-path prefill would quantise its activations
    # per token, which the oracle then mirrors on the prompt rows
    fused = eng_fused
    bad_pos = checked = 0
    for p, g in zip(_prompts(), got):
        ids = list(p)
        for t in g:
            lg = dense_logits_fp8(m1, ids, 0 if fused else len(p))
            checked += 1
            if int(torch.argmax(lg)) != t:
                gap = float(lg.max() - lg[t])
                assert gap < 0.3, (g, len(ids) - len(p), gap)
                bad_pos += 1
            ids.append(t)
    assert bad_pos <= checked // 5, (bad_pos, checked, got, exp)


def _ipc_ar_worker(rank, world, port, q):
    try:
        from agentic_traffic_testing_amd.parallel.comm import init_distributed
        from agentic_traffic_testing_amd.parallel.custom_allreduce import IpcAllReduce

        torch.cuda.set_device(0)
        comm = init_distributed(rank, world, "cuda:0", "gloo", "127.0.0.1", port)
        ar = IpcAllReduce(comm, "cuda:0", max_bytes=16 * 8192 * 2,
                          large_max_bytes=512 * 8192 * 2)
        bad = []
        sizes = [8, 7, 4096, 8192 * 5 + 3, 16 * 8192, 1000, 4096, 300 * 8192 + 5, 512 * 8192]
        for it, n in enumerate(sizes * 4):
            g = torch.Generator(device="cpu").manual_seed(1000 * it)
            parts = [torch.randn(n, generator=g).to(torch.bfloat16) for _ in range(world)]
            exp = torch.zeros(n)
            for p_ in parts:  # rank order, fp32, like the kernels
                exp += p_.float()
            exp = exp.to(torch.bfloat16)
            # auto policy, then both kernels explicitly where the message fits them
            modes = ["auto"] + (["oneshot"] if n <= ar.max_elems else []) + ["twoshot"]
            for mode in modes:
                x = parts[rank].cuda()
                ar.all_reduce(x, mode)
                torch.cuda.synchronize()
                if not torch.equal(x.cpu(), exp):
                    bad.append((it, n, mode))
        # graph-captured replays with fresh inputs each time
        x = torch.empty(4096, dtype=torch.bfloat16, device="cuda")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            ar.all_reduce(x.fill_(1.0))
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        xl = torch.empty(200 * 8192, dtype=torch.bfloat16, device="cuda")
        with torch.cuda.stream(s):
            ar.all_reduce(xl.fill_(1.0), "twoshot")
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        with torch.cuda.graph(graph):
            ar.all_reduce(x)
            ar.all_reduce(xl, "twoshot")
        for k in range(5):
            x.fill_(float(rank + k))
            xl.fill_(float(2 * rank - k))
            graph.replay()
            torch.cuda.synchronize()
            want = float(sum(r + k for r in range(world)))
            if not bool((x == want).all()):
                bad.append(("graph", k, float(x[0])))
            want2 = float(sum(2 * r - k for r in range(world)))
            if not bool((xl == want2).all()):
                bad.append(("graph2", k, float(xl[0])))
        if ar.check() != 0:
            bad.append(("timeout-word", ar.check()))
        comm.barrier()
        ar.close()
        q.put((rank, bad, ar.calls))
        torch.distributed.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), -1))


def _ipc_push_worker(rank, world, port, q):
    try:
        from agentic_traffic_testing_amd import ops
        from agentic_traffic_testing_amd.parallel.comm import init_distributed
        from agentic_traffic_testing_amd.parallel.custom_allreduce import IpcAllReduce

        torch.cuda.set_device(0)
        comm = init_distributed(rank, world, "cuda:0", "gloo", "127.0.0.1", port)
        ar = IpcAllReduce(comm, "cuda:0", max_bytes=16 * 8192 * 2)
        bad = []
        for it, (B, N, K) in enumerate([(1, 4096, 1024), (5, 8192, 1024), (16, 4096, 512),
                                        (3, 4096, 3584)] * 3):
            g = torch.Generator(device="cpu").manual_seed(100 * it + rank)
            x = torch.randn(B, K, generator=g).to(torch.bfloat16).cuda()
            w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).cuda()
            gr = torch.Generator(device="cpu").manual_seed(7 + it)  # same residual everywhere
            res = torch.randn(B, N, generator=gr).to(torch.bfloat16).cuda()
            # reference: the unfused path (GEMV, then the one-shot kernel with the residual add)
            r1 = res.clone()
            ar.all_reduce(ops.linear(x, w), residual=r1)
            # fused push: the GEMV epilogue pushes, one receive kernel adds the sum
            r2 = res.clone()
            ops.linear_push_reduce(x, w, r2, ar)
            torch.cuda.synchronize()
            if not torch.equal(r1, r2):
                bad.append((it, B, N, K, float((r1.float() - r2.float()).abs().max())))
        # graph-captured replays of the push path with fresh inputs each time
        B, N, K = 4, 4096, 1024
        x = torch.empty(B, K, dtype=torch.bfloat16, device="cuda")
        w = (torch.randn(N, K, device="cuda") / 32).to(torch.bfloat16)
        r = torch.empty(B, N, dtype=torch.bfloat16, device="cuda")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            ops.linear_push_reduce(x.fill_(0.5), w, r.fill_(0.0), ar)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            ops.linear_push_reduce(x, w, r, ar)
        for k in range(4):
            x.copy_(torch.full((B, K), 0.25 * (rank + k + 1), device="cuda").to(torch.bfloat16))
            r.fill_(1.0)
            graph.replay()
            torch.cuda.synchronize()
            exp = r.clone().fill_(1.0)
            ar.all_reduce(ops.linear(x, w), residual=exp)
            torch.cuda.synchronize()
            if not torch.equal(r, exp):
                bad.append(("graph", k))
        if ar.check() != 0:
            bad.append(("timeout-word", ar.check()))
        comm.barrier()
        ar.close()
        q.put((rank, bad, ar.calls_push))
        torch.distributed.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), -1))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_ipc_fused_push_matches_oneshot(world):
    """X1 / X2 with the push fused into the row-parallel GEMV (skinny.h push epilogue +
    allreduce.hip push_reduce_kernel) is bit-identical to GEMV + one-shot kernel at 2 / 4 / 8
    ranks on one MI355X, eager and graph-replayed, mixed with one-shot calls on one buffer."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_ipc_push_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for rank, bad, calls in res:
        assert bad == [], bad
        assert calls > 10


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_ipc_allreduce_ranks_one_gpu(world):
    """One-shot and two-shot IPC all-reduce at 2 / 4 / 8 ranks (all on one MI355X): exact
    fp32 rank-order sums for odd and prefill-sized messages, graph-captured replays."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_ipc_ar_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for rank, bad, calls in res:
        assert bad == [], bad
        assert calls > 20


@pytest.mark.gpu
@pytest.mark.parametrize("tp", [1, 8])
def test_fp8_fused_past_32_rows_prefill_and_decode(tp):
    """fp8 weights (BASELINE config 5) on the fused kernels past 32 rows, TP=1
    and a same-GPU TP=8 rehearsal on the 70B per-rank geometry: one 96-row prefill step of 48
    sequences (wide kernel W8 builds: norm fold + RoPE / KV write, SiLU-mul, and o / down whose
    partial sums take the IPC all-reduce - past the fused push's 32 rows) and B=48 decode steps
    replayed from hipGraphs.  Tokens teacher-forced against the fp32 oracle of the dequantised
    weights with 16-bit activations (weight-only, like the kernels), near-tie rule."""
    from helpers import dense_logits_fp8

    rng = np.random.default_rng(17)
    prompts = [rng.integers(300, 3000, size=n).tolist() for n in [2] * 48]
    base = dict(model="llama-70b-tp-slice-fp8", device="cuda:0", max_model_len=256,
                num_kv_blocks=256, max_num_batched_tokens=512, max_num_seqs=48,
                graph_batch_sizes=(1, 8, 48), use_graphs=True, quantization="fp8")
    greedy = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True)
    ref_eng = LLMEngine(EngineConfig(**base))
    m1 = ref_eng.runner.model
    if tp == 1:
        eng = ref_eng
    else:
        eng = TPEngine(EngineConfig(tensor_parallel_size=tp, tp_same_device=True,
                                    tp_allreduce="ipc", tp_fused_push=True, **base))
    try:
        r = eng.runner
        m = r.model
        assert m.quant == "fp8" and m.small_prefill_ok(96) and m.decode_fusable(48)
        assert not m.midm_route(96) and not m.midm_fp8_ok(96)
        steps0, g0 = r.steps, r.graph_steps
        got = [o.token_ids for o in eng.generate(prompts, greedy)]
        assert all(len(g) == 6 for g in got)
        decode_steps = r.steps - steps0 - 1
        assert r.graph_steps - g0 >= 0.8 * decode_steps, (r.graph_steps - g0, decode_steps)
        if tp > 1:
            assert eng.comm.ipc.check() == 0
    finally:
        if tp > 1:
            eng.shutdown()
    bad_pos = checked = 0
    for p, g in list(zip(prompts, got))[::4]:
        ids = list(p)
        for t in g:
            lg = dense_logits_fp8(m1, ids, 0)
            checked += 1
            if int(torch.argmax(lg)) != t:
                gap = float(lg.max() - lg[t])
                assert gap < 0.3, (g, len(ids) - len(p), gap)
                bad_pos += 1
            ids.append(t)
    assert bad_pos <= checked // 5, (bad_pos, checked)
