"""One-shot IPC all-reduce for small TP messages.

Wraps ops/csrc/allreduce.hip: every rank allocates one uncached, IPC-exportable device
buffer, the buffers' IPC handles are exchanged once over the process group
(``all_gather_object``), and each rank maps its peers' buffers.  ``all_reduce(x)`` then
runs ONE kernel that pushes x's slices into every peer over xGMI, flags them, and sums the
incoming copies locally in rank order (bit-identical on every rank) - no RCCL ring, no
host involvement, hipGraph-capturable.  Messages above ``max_bytes`` (prefill) stay on
RCCL via ``TPComm``.

Selected with ``EngineConfig.tp_allreduce = "ipc"``.  Requires HSA_ENABLE_IPC_MODE_LEGACY=0
(dmabuf IPC) like every cross-process device-memory share on this stack.  Ranks may share
one GPU (the single-GPU test rehearsal) - the protocol is the same.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class IpcAllReduce:
    def __init__(self, comm, device, max_bytes: int, dtype=torch.bfloat16):
        if comm.size not in (2, 4, 8):
            raise ValueError("IPC all-reduce supports 2, 4 or 8 ranks")
        self.comm = comm
        self.device = torch.device(device)
        self.elem = torch.finfo(dtype).bits // 8
        self.max_elems = max(8, (max_bytes // self.elem + 7) // 8 * 8)
        from ..ops import _native

        ops = self._ops = _native()  # loads the kernel library (fails loudly if absent)
        nbytes = ops.ar_buffer_bytes(self.max_elems, self.elem)
        self.local = ops.ar_alloc(nbytes, self.device.index or 0)
        handle = ops.ar_handle(self.local).tolist()
        handles = [None] * comm.size
        dist.all_gather_object(handles, handle, group=comm.group)
        self.bases = []
        self.opened = []
        for r, h in enumerate(handles):
            if r == comm.rank:
                self.bases.append(self.local)
            else:
                p = ops.ar_open(torch.tensor(h, dtype=torch.uint8))
                self.opened.append(p)
                self.bases.append(p)
        comm.barrier()  # every rank mapped every buffer before the first kernel
        self.calls = 0

    def eligible(self, x: torch.Tensor) -> bool:
        return (x.is_cuda and x.is_contiguous() and x.dtype in (torch.bfloat16, torch.float16)
                and 0 < x.numel() <= self.max_elems)

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        self._ops.ar_run(x, x, self.bases, self.comm.rank, self.max_elems)
        self.calls += 1
        return x

    def check(self) -> int:
        """Error word of the local buffer: bit q set = a wait for rank q timed out."""
        return int(self._ops.ar_error(self.local))

    def close(self):
        ops = self._ops
        for p in self.opened:
            ops.ar_close(p)
        self.opened = []
        if self.local:
            torch.cuda.synchronize(self.device)
            ops.ar_free(self.local)
            self.local = 0
