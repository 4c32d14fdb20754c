"""ROCTx ranges around the serving engine's host phases (SURVEY §5.1 tracing/profiling).

``ATTA_ROCTX=1`` turns them on: the engine then brackets scheduling, step launch, token
collection and synchronous steps with ``roctxRangePushA`` / ``roctxRangePop`` from
rocprofiler-sdk's ROCTx library, so ``rocprofv3 --marker-trace --kernel-trace`` shows the
host phases on the same timeline as the kernels (which ranges a hipGraph replay or a prefill
GEMM sits in).  Off (default) every call is a no-op: no library load, no per-step cost.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_LIBS = ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
         "libroctx64.so")
_lib = None
ENABLED = os.environ.get("ATTA_ROCTX", "0") == "1"


def _load():
    global _lib, ENABLED
    if _lib is not None or not ENABLED:
        return _lib
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    for name in _LIBS:
        for cand in (os.path.join(rocm, "lib", name), name):
            try:
                lib = ctypes.CDLL(cand)
            except OSError:
                continue
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _lib = lib
            return _lib
    ENABLED = False  # no ROCTx library: stay a no-op
    return None


def push(name: str) -> None:
    if ENABLED and _load() is not None:
        _lib.roctxRangePushA(name.encode())


def pop() -> None:
    if ENABLED and _lib is not None:
        _lib.roctxRangePop()


def mark(name: str) -> None:
    if ENABLED and _load() is not None:
        _lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors the ROCTx API name
    if not ENABLED:
        yield
        return
    push(name)
    try:
        yield
    finally:
        pop()
