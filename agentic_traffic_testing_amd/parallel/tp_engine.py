"""Tensor-parallel serving engine: one process per GPU, rank 0 serves.

The reference cannot run tensor parallelism (``tensor_parallel_size`` in
llm/config/llama-3.1-8b.yaml:2 is never read; vLLM is built with its defaults at
llm/serve_llm.py:362-378).  Here TP is first-class and MI355X-shaped:

* rank r owns GPU r (``cuda:r``), one OS process each, joined by a ``torch.distributed``
  group whose ``"nccl"`` backend is RCCL over the node's point-to-point xGMI links;
* rank 0 runs the HTTP front end, scheduler and block manager; each step it publishes the
  packed int32 step metadata on a shared-memory channel (runtime ShmChannel) and every
  rank then runs the identical kernel + all-reduce sequence (``ModelRunner.serve_worker``);
* decode steps are hipGraph-captured on every rank (RCCL kernels inside the graph);
* sampling is vocab-parallel with a single int64 MAX all-reduce per step (parallel/comm.py).

Launch modes:

* ``TPEngine(cfg)`` from a plain process spawns ranks 1..N-1 with ``multiprocessing``
  (spawn) before this process touches the GPU;
* under ``torchrun --nproc-per-node N`` (RANK / WORLD_SIZE set) rank 0 builds
  ``TPEngine(cfg, external=True)`` and the other ranks call ``run_worker``.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import socket
import time

import torch

from ..config import EngineConfig, resolve_model
from ..engine.llm_engine import LLMEngine
from ..engine.model_runner import HDR_WORDS, ModelRunner
from .comm import init_distributed


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def channel_name(port: int) -> str:
    return f"atta_tp_{port}"


def rank_device(cfg: EngineConfig, rank: int) -> str:
    dev = torch.device(cfg.device)
    if dev.type != "cuda":
        return "cpu"
    if cfg.tp_same_device:
        return f"cuda:{dev.index or 0}"
    return f"cuda:{rank}"


def _attach(name: str, timeout_s: float = 600.0):
    from ..runtime import ShmChannel

    t0 = time.monotonic()
    while True:
        try:
            return ShmChannel(name, create=False)
        except RuntimeError:
            if time.monotonic() - t0 > timeout_s:
                raise
            time.sleep(0.05)


def run_worker(cfg: EngineConfig, rank: int, world: int, port: int) -> None:
    """Body of TP rank > 0: build the shard, then replay rank 0's steps until stopped."""
    device = rank_device(cfg, rank)
    comm = init_distributed(rank, world, device, _backend(cfg), "127.0.0.1", port)
    mcfg, wdir = resolve_model(cfg.model)
    runner = ModelRunner(cfg, mcfg, device, comm=comm, weights_dir=wdir)
    _maybe_ipc(cfg, comm, runner)
    ch = _attach(channel_name(port))
    try:
        runner.serve_worker(ch, rank - 1)
    finally:
        if torch.distributed.is_initialized():
            torch.distributed.destroy_process_group()


def _spawned_worker(cfg_dict: dict, rank: int, world: int, port: int) -> None:
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    run_worker(EngineConfig(**cfg_dict), rank, world, port)


def _backend(cfg: EngineConfig) -> str:
    if cfg.tp_backend != "auto":
        return cfg.tp_backend
    if torch.device(cfg.device).type != "cuda" or cfg.tp_same_device:
        return "gloo"  # RCCL refuses two ranks on one device
    return "nccl"


def _maybe_ipc(cfg: EngineConfig, comm, runner: ModelRunner):
    """Install the custom IPC all-reduce (one-shot for decode-sized messages, two-shot up to
    a prefill chunk): always with tp_allreduce="ipc", and with "auto" when the ranks sit on
    distinct GPUs of the node (RCCL backend) - the xGMI case it is built for."""
    if comm.size == 1 or not runner.is_cuda or comm.size not in (2, 4, 8):
        return
    if cfg.tp_allreduce == "rccl":
        return
    if cfg.tp_allreduce == "auto" and (comm.is_gloo or cfg.tp_same_device):
        return
    from .custom_allreduce import IpcAllReduce

    H = runner.mcfg.hidden_size
    comm.ipc = IpcAllReduce(comm, runner.device, max_bytes=runner.max_seqs * H * 2,
                            large_max_bytes=min(cfg.max_num_batched_tokens, 8192) * H * 2)
    comm.fused_push = bool(getattr(cfg, "tp_fused_push", True))


class TPEngine(LLMEngine):
    def __init__(self, cfg: EngineConfig, external: bool = False):
        world = cfg.tensor_parallel_size
        if world < 2:
            raise ValueError("TPEngine needs tensor_parallel_size >= 2")
        self.procs: list = []
        port = int(os.environ.get("MASTER_PORT", "29511")) if external else (
            cfg.dist_port or free_port())
        # drop a stale segment of a crashed earlier run before any worker can attach to it
        # (workers attach only after the first collective, which needs this rank)
        stale = f"/dev/shm/{channel_name(port)}"
        if os.path.exists(stale):
            os.remove(stale)
        if not external:
            ctx = mp.get_context("spawn")
            for r in range(1, world):
                p = ctx.Process(target=_spawned_worker, args=(cfg.as_dict(), r, world, port),
                                name=f"atta-tp-rank{r}", daemon=True)
                p.start()
                self.procs.append(p)
        device = rank_device(cfg, 0)
        comm = init_distributed(0, world, device, _backend(cfg), "127.0.0.1", port)
        self.comm = comm
        mcfg, wdir = resolve_model(cfg.model)
        runner = ModelRunner(cfg, mcfg, device, comm=comm, weights_dir=wdir)
        _maybe_ipc(cfg, comm, runner)
        from ..runtime import ShmChannel

        # workers poll for the channel after their own (identical) runner init; a worker
        # that has not registered within tp_register_timeout_s counts as dead (it died
        # before it could register, e.g. out of memory while loading its shard)
        self.channel = ShmChannel(channel_name(port), HDR_WORDS + runner.max_layout.size,
                                  world - 1, create=True,
                                  register_timeout_s=cfg.tp_register_timeout_s)
        runner.publisher = self.channel
        self._defer_warmup = True
        super().__init__(cfg, runner=runner, device=device)
        self._closed = False
        try:
            runner.capture_all()
            if cfg.startup_warmup and runner.is_cuda:
                self.warmup()
        except BaseException:
            self.kill()
            raise

    # a step that raises after rank 0 published it leaves the workers inside collectives
    # rank 0 never joins: the serving loop must stop the group instead of continuing
    step_failure_fatal = True

    def kill(self):
        """Stop the TP group without the stop handshake (used after a failed step):
        close the step channel so idle workers exit, terminate spawned workers that are
        stuck in a collective, and tear down the process group."""
        if getattr(self, "_closed", True):
            return
        self._closed = True
        ch = getattr(self, "channel", None)
        if ch is not None:
            ch.close()
        for p in self.procs:
            p.join(timeout=2)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
        try:
            if torch.distributed.is_initialized():
                torch.distributed.destroy_process_group()
        except Exception:
            pass

    def dead_ranks(self) -> list[int]:
        """TP ranks whose process is gone (spawned children, or torchrun peers that had
        registered on the step channel) - SURVEY §5.3 TP-rank liveness."""
        dead = {i + 1 for i, p in enumerate(self.procs) if not p.is_alive()}
        ch = getattr(self, "channel", None)
        if ch is not None:
            dead.update(r + 1 for r in ch.dead_readers())
        return sorted(dead)

    def shutdown(self):
        if getattr(self, "_closed", True):
            return
        self._closed = True
        try:
            self.runner.stop_workers()
        finally:
            for p in self.procs:
                p.join(timeout=60)
                if p.is_alive():
                    p.terminate()
            if torch.distributed.is_initialized():
                torch.distributed.destroy_process_group()

    def __del__(self):
        try:
            self.shutdown()
        except Exception:
            pass
