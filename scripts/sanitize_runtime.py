"""Stress the native host runtime (block manager + TP step channel) under ASan/UBSan.

Run by tests/test_sanitizers.py as
    LD_PRELOAD=<libasan.so> ASAN_OPTIONS=detect_leaks=0 python scripts/sanitize_runtime.py
against the sanitized build (ops/build.py build_runtime_sanitized).  Any heap overflow,
use-after-free or undefined behaviour in the C++ aborts the process with a report.
"""
import importlib.util
import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(path):
    spec = importlib.util.spec_from_file_location("_atta_runtime", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def block_manager_stress(rt, seed=0, rounds=3000):
    rng = np.random.default_rng(seed)
    bs = 16
    bm = rt.BlockManager(96, bs, True)
    live = {}
    next_id = 1
    shared = rng.integers(0, 1000, size=64).astype(np.int64)
    for _ in range(rounds):
        op = rng.integers(0, 5)
        if op <= 1 and len(live) < 12:  # admit (half the prompts share a cached prefix)
            n = int(rng.integers(1, 120))
            toks = rng.integers(0, 1000, size=n).astype(np.int64)
            if rng.random() < 0.5:
                toks[:min(n, 64)] = shared[:min(n, 64)]
            cached = bm.allocate(next_id, toks, n + 1)
            if cached >= 0:
                live[next_id] = [toks, int(cached)]
                next_id += 1
        elif op == 2 and live:  # grow a sequence by one decode token
            sid = int(rng.choice(list(live)))
            toks, done = live[sid]
            toks = np.append(toks, rng.integers(0, 1000)).astype(np.int64)
            if bm.ensure(sid, len(toks)):
                live[sid] = [toks, len(toks) - 1]
                bm.commit(sid, toks, len(toks) - 1)
        elif op == 3 and live:  # build a step's metadata (decode rows + prefill tiles)
            ids = np.array(list(live)[:8], dtype=np.int64)
            qs = np.array([max(0, live[i][1] - 3) for i in ids], dtype=np.int64)
            ql = np.array([len(live[i][0]) - q for i, q in zip(ids, qs)], dtype=np.int64)
            ql = np.maximum(ql, 1)
            try:
                d = bm.build_batch(ids, qs, ql, 16, 32, 0, 4, len(ids) + 2)
                assert d["positions"].shape[0] >= int(ql.sum())
            except (ValueError, RuntimeError, IndexError):
                pass  # rejected shapes must raise, never corrupt memory
        elif live:  # finish
            sid = int(rng.choice(list(live)))
            bm.free(sid)
            del live[sid]
    for sid in list(live):
        bm.free(sid)
    assert bm.num_free_blocks() == 96


def _reader(path, name, r, n_msgs, q):
    rt = load(path)
    ch = rt.ShmChannel(name)
    ch.register_reader(r)
    last, got = 0, 0
    while got < n_msgs:
        msg = ch.receive(r, last, 5.0)
        if msg is None:
            break
        last, data = msg
        assert int(data[0]) == last and data.shape[0] == 1 + (last % 37)
        got += 1
    q.put(got)


def channel_stress(rt, path, n_readers=3, n_msgs=2000):
    name = f"atta-asan-{os.getpid()}"
    ch = rt.ShmChannel(name, 64, n_readers, True, 30.0)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_reader, args=(path, name, r, n_msgs, q)) for r in range(n_readers)]
    for p in ps:
        p.start()
    for i in range(1, n_msgs + 1):
        ch.publish(np.full(1 + (i % 37), i, dtype=np.int32), 30.0)
    got = [q.get(timeout=60) for _ in ps]
    for p in ps:
        p.join(30)
    ch.close()
    assert got == [n_msgs] * n_readers, got
    try:  # oversize messages are rejected, not copied past the slot
        ch.publish(np.zeros(65, dtype=np.int32), 1.0)
        raise AssertionError("oversize publish accepted")
    except (ValueError, RuntimeError, IndexError):
        pass


if __name__ == "__main__":
    path = sys.argv[1]
    rt = load(path)
    block_manager_stress(rt)
    channel_stress(rt, path)
    print("SANITIZED RUNTIME OK")
