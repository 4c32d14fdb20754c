"""Tensor-parallel communication primitives.

The reference has no GPU collectives at all ("In the reference: none"); this
module is the MI355X build's comm layer for Megatron-style TP inside one node:

* ``TPComm`` wraps one ``torch.distributed`` process group.  On GPUs the backend is
  ``"nccl"``, which is RCCL on ROCm, riding the 7 point-to-point xGMI links of an MI355X
  node; the CPU test path (and a single-GPU multi-process rehearsal) uses ``gloo``.
* X1/X2 ``all_reduce`` after the row-parallel o_proj / down_proj.  Decode messages are
  tiny ([B, hidden] bf16 = B x 8-16 KiB), latency-bound; they are issued on the compute
  stream so a decode step captured into a hipGraph contains the RCCL kernels too.
  ``IpcAllReduce`` (ops/csrc/allreduce.hip) can replace RCCL for those small messages.
* X4 sampling across the vocab shards: each rank reduces its shard to one packed int64
  (score, -id) key per row and a single int64 MAX all-reduce picks the global winner, so
  no [B, V/tp] logits all-gather is needed on the fused decode path.
* ``all_gather_last`` (prefill / unfused logits) concatenates vocab shards.

gloo has no bf16/fp16 reduction kernels on some builds, so gloo reductions run in fp32;
gloo collectives on device tensors (several ranks rehearsing on ONE GPU, where RCCL refuses
duplicate devices) are staged through host memory.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class TPComm:
    rank: int
    size: int
    group: object = None          # torch.distributed ProcessGroup (None = default group)
    backend: str = "nccl"
    ipc: object = None            # optional IpcAllReduce for small messages

    @property
    def is_gloo(self) -> bool:
        return self.backend == "gloo"

    # -- X1 / X2 ------------------------------------------------------------------------
    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        if self.size == 1:
            return x
        if self.ipc is not None and self.ipc.eligible(x):
            return self.ipc.all_reduce(x)
        if self.is_gloo:
            return self._gloo_inplace(x, dist.ReduceOp.SUM)
        dist.all_reduce(x, group=self.group)
        return x

    def all_reduce_residual(self, x: torch.Tensor, residual: torch.Tensor) -> torch.Tensor:
        """``residual += all_reduce(x)`` (row-parallel o / down projections).  On the IPC
        path the add is the reduction kernel's epilogue: no extra launch or HBM pass."""
        if self.size == 1:
            return residual.add_(x)
        if self.ipc is not None and self.ipc.eligible(x):
            return self.ipc.all_reduce(x, residual=residual)
        return residual.add_(self.all_reduce(x))

    def push_ok(self, rows: int, n_out: int) -> bool:
        """Can a row-parallel decode GEMV push its product straight into the peers'
        receive slots (IPC path, fused push)?"""
        return (self.size > 1 and self.ipc is not None and self.fused_push
                and rows <= 32 and self.ipc.push_eligible(rows, n_out))  # GEMV: <= 32 rows

    fused_push: bool = True

    @property
    def decode_capturable(self) -> bool:
        """Can a decode step's collectives (X1/X2 sums, X4 key MAX) be hipGraph-captured?
        RCCL: yes.  gloo (a same-GPU rehearsal's control group): only when the IPC kernels
        carry them - then the whole step stays on the device."""
        return self.size == 1 or not self.is_gloo or self.ipc is not None

    def _gloo_inplace(self, x: torch.Tensor, op) -> torch.Tensor:
        tmp = x.float() if x.dtype in (torch.bfloat16, torch.float16) else x
        tmp = tmp.cpu() if tmp.is_cuda else tmp
        if tmp.data_ptr() == x.data_ptr():
            tmp = tmp.clone() if not tmp.is_contiguous() else tmp
        dist.all_reduce(tmp, op=op, group=self.group)
        if tmp.data_ptr() != x.data_ptr():
            x.copy_(tmp)
        return x

    # -- X4 ---------------------------------------------------------------------------------
    def all_reduce_max(self, x: torch.Tensor, tokens: torch.Tensor | None = None) -> torch.Tensor:
        """In-place MAX.  For sampler keys with ``tokens``, the decoded winners are written
        there too (IPC path: by the reduction kernel itself)."""
        if self.size == 1:
            pass
        elif self.ipc is not None and self.ipc.keys_eligible(x):
            return self.ipc.all_reduce_max_keys(x, tokens)
        elif self.is_gloo:
            self._gloo_inplace(x, dist.ReduceOp.MAX)
        else:
            dist.all_reduce(x, op=dist.ReduceOp.MAX, group=self.group)
        if tokens is not None:
            tokens[:x.shape[0]].copy_(0xFFFFFFFF - (x & 0xFFFFFFFF))
        return x

    def all_gather_last(self, x: torch.Tensor) -> torch.Tensor:
        if self.size == 1:
            return x
        src = x
        if self.is_gloo:
            src = x.float() if x.dtype in (torch.bfloat16, torch.float16) else x
            src = src.cpu()
        parts = [torch.empty_like(src) for _ in range(self.size)]
        dist.all_gather(parts, src.contiguous(), group=self.group)
        return torch.cat(parts, dim=-1).to(device=x.device, dtype=x.dtype)

    # -- X6 ---------------------------------------------------------------------------------
    def min_int(self, v: int, device) -> int:
        if self.size == 1:
            return int(v)
        dev = torch.device("cpu") if self.is_gloo else torch.device(device)
        t = torch.tensor([int(v)], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return int(t.item())

    def barrier(self):
        if self.size > 1:
            dist.barrier(group=self.group)


def init_distributed(rank: int, world: int, device: str, backend: str = "auto",
                     master_addr: str | None = None, master_port: int | None = None) -> TPComm:
    """Initialise the default process group for one TP rank (idempotent)."""
    dev = torch.device(device)
    if backend == "auto":
        backend = "nccl" if dev.type == "cuda" else "gloo"
    if world == 1:
        return TPComm(rank=0, size=1, backend=backend)
    os.environ.setdefault("MASTER_ADDR", master_addr or "127.0.0.1")
    if master_port:
        os.environ["MASTER_PORT"] = str(master_port)
    os.environ.setdefault("MASTER_PORT", "29511")
    if not dist.is_initialized():
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(dev)
            kw["device_id"] = dev
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return TPComm(rank=rank, size=world, group=None, backend=backend)


# Legacy functional API used by models/llama.py --------------------------------------------
_DEFAULT: TPComm | None = None


def set_default(comm: TPComm | None):
    global _DEFAULT
    _DEFAULT = comm


def tp_all_reduce(x: torch.Tensor, comm: TPComm | None = None) -> torch.Tensor:
    c = comm or _DEFAULT
    return x if c is None else c.all_reduce(x)


def tp_all_gather_last(x: torch.Tensor, comm: TPComm | None = None) -> torch.Tensor:
    c = comm or _DEFAULT
    return x if c is None else c.all_gather_last(x)
