"""Custom intra-node all-reduce over IPC-mapped peer buffers.

Wraps ops/csrc/allreduce.hip.  Every rank allocates uncached, IPC-exportable device buffers;
their IPC handles are exchanged once over the process group (``all_gather_object``) and each
rank maps its peers' buffers.  Two kernels, both hipGraph-capturable (all state on the
device, fixed grids, kernel arguments never change):

* **one-shot** (decode-sized messages, [B, hidden] bf16 = 8 KiB - 256 KiB): every rank PUSHES
  its whole input into every peer over the point-to-point xGMI links (one hop, all links busy
  at once) and sums the W copies locally in rank order - latency-optimal.
* **two-shot** (prefill-sized messages): reduce-scatter (rank q receives everyone's copy of
  chunk q and sums it) then all-gather (rank q pushes its reduced chunk to everyone) - every
  rank moves 2 (W-1)/W of the message over its links instead of (W-1) whole copies, the
  bandwidth-optimal shape of a ring in 2 hops instead of 2 (W-1).

Both sum in fp32 in rank order, so every rank gets bit-identical results and the two kernels
agree with each other.  Messages above the two-shot buffer stay on RCCL (``TPComm``).

Selected with ``EngineConfig.tp_allreduce``: "ipc" always, "auto" whenever the TP ranks sit
on distinct GPUs of one node (RCCL backend).  Requires HSA_ENABLE_IPC_MODE_LEGACY=0 (dmabuf
IPC) like every cross-process device-memory share on this stack.  Ranks may share one GPU
(the single-GPU test rehearsal) - the protocol is the same.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

# one-shot up to this many bytes, two-shot above (xGMI: one hop of W-1 full copies stops
# paying once the per-link bytes dominate the ~2 extra hand-off latencies of two-shot)
ONESHOT_MAX_BYTES = int(os.environ.get("ATTA_AR_ONESHOT_MAX", str(512 << 10)))


class _PeerBuffers:
    """One uncached device buffer per rank, mapped into every rank."""

    def __init__(self, ops, comm, device, nbytes: int):
        self.ops = ops
        self.device = device
        self.local = ops.ar_alloc(nbytes, device.index or 0)
        handle = ops.ar_handle(self.local).tolist()
        handles = [None] * comm.size
        dist.all_gather_object(handles, handle, group=comm.group)
        self.bases, self.opened = [], []
        for r, h in enumerate(handles):
            if r == comm.rank:
                self.bases.append(self.local)
            else:
                p = ops.ar_open(torch.tensor(h, dtype=torch.uint8))
                self.opened.append(p)
                self.bases.append(p)

    def close(self):
        for p in self.opened:
            self.ops.ar_close(p)
        self.opened = []
        if self.local:
            torch.cuda.synchronize(self.device)
            self.ops.ar_free(self.local)
            self.local = 0


class IpcAllReduce:
    def __init__(self, comm, device, max_bytes: int, dtype=torch.bfloat16,
                 large_max_bytes: int = 0):
        """``max_bytes``: largest one-shot message; ``large_max_bytes`` (> 0): also map
        two-shot buffers for messages up to that size."""
        if comm.size not in (2, 4, 8):
            raise ValueError("IPC all-reduce supports 2, 4 or 8 ranks")
        self.comm = comm
        self.device = torch.device(device)
        self.elem = torch.finfo(dtype).bits // 8
        self.max_elems = max(8, (max_bytes // self.elem + 7) // 8 * 8)
        from ..ops import _native

        ops = self._ops = _native()  # loads the kernel library (fails loudly if absent)
        self.small = _PeerBuffers(ops, comm, self.device,
                                  ops.ar_buffer_bytes(self.max_elems, self.elem))
        self.bases = self.small.bases
        self.local = self.small.local
        self.large = None
        self.max_elems2 = 0
        if large_max_bytes > 0:
            self.max_elems2 = max(8, (large_max_bytes // self.elem + 7) // 8 * 8)
            self.large = _PeerBuffers(ops, comm, self.device,
                                      ops.ar2_buffer_bytes(self.max_elems2, comm.size,
                                                           self.elem))
        comm.barrier()  # every rank mapped every buffer before the first kernel
        self.calls = 0
        self.calls2 = 0
        self.calls_max = 0
        self.calls_push = 0

    def _ok(self, x: torch.Tensor) -> bool:
        return (x.is_cuda and x.is_contiguous() and x.dtype in (torch.bfloat16, torch.float16)
                and x.numel() > 0)

    def eligible(self, x: torch.Tensor) -> bool:
        return self._ok(x) and (x.numel() <= self.max_elems or x.numel() <= self.max_elems2)

    def all_reduce(self, x: torch.Tensor, mode: str = "auto",
                   residual: torch.Tensor | None = None) -> torch.Tensor:
        """Sum over the TP ranks, in place in ``x`` - or, with ``residual``, the residual-stream
        update ``residual += sum`` fused into the reduction's epilogue (returns residual).
        ``mode``: auto | oneshot | twoshot."""
        n = x.numel()
        y = x if residual is None else residual
        two = mode == "twoshot" or (mode == "auto" and (
            n > self.max_elems or n * self.elem > ONESHOT_MAX_BYTES) and n <= self.max_elems2)
        if two:
            if self.large is None or n > self.max_elems2:
                raise ValueError("message larger than the two-shot buffer")
            self._ops.ar2_run(x, y, self.large.bases, self.comm.rank, self.max_elems2, residual)
            self.calls2 += 1
        else:
            if n > self.max_elems:
                raise ValueError("message larger than the one-shot buffer")
            self._ops.ar_run(x, y, self.bases, self.comm.rank, self.max_elems, residual)
            self.calls += 1
        return y

    # -- X1 / X2 with the push fused into the row-parallel GEMV ------------------------------
    def push_eligible(self, rows: int, n_out: int) -> bool:
        return rows * n_out <= self.max_elems and n_out % 16 == 0

    def gemv_push(self, x: torch.Tensor, w: torch.Tensor, n_out: int, waves: int,
                  preshuffled: bool, w_scale, ksplit: int) -> None:
        """Row-parallel decode GEMV whose epilogue writes x @ w.T of this rank's K shard
        straight into every rank's receive slot (no local output, no separate push);
        ``push_reduce`` completes the all-reduce."""
        self._ops.skinny_gemm_push(x, w, n_out, waves, preshuffled, w_scale, ksplit,
                                   self.bases, self.comm.rank, self.max_elems)

    def push_reduce(self, residual: torch.Tensor, n_out: int) -> torch.Tensor:
        """residual += sum over ranks of the pushed products (rank-order fp32 sum, the
        residual add in the same kernel); n_out / 16 tiles were pushed by every source."""
        self._ops.ar_push_reduce(residual, residual, self.bases, self.comm.rank,
                                 self.max_elems, n_out // 16)
        self.calls_push += 1
        return residual

    MAX_KEYS = 256

    def keys_eligible(self, keys: torch.Tensor) -> bool:
        return (keys.is_cuda and keys.is_contiguous() and keys.dtype == torch.int64
                and 0 < keys.numel() <= self.MAX_KEYS)

    def all_reduce_max_keys(self, keys: torch.Tensor,
                            tokens: torch.Tensor | None = None) -> torch.Tensor:
        """X4: in-place int64 MAX of the vocab-parallel sampler keys over the TP ranks (one
        tiny kernel on the one-shot peer buffers); with ``tokens`` the winners' token ids are
        written there by the same kernel."""
        self._ops.ar_keymax(keys, tokens, self.bases, self.comm.rank)
        self.calls_max += 1
        return keys

    def check(self) -> int:
        """Error words: bit q set = a wait for rank q timed out (one-shot | two-shot)."""
        err = int(self._ops.ar_error(self.small.local))
        if self.large is not None:
            err |= int(self._ops.ar2_error(self.large.local))
        return err

    def close(self):
        self.small.close()
        if self.large is not None:
            self.large.close()
        self.local = 0
