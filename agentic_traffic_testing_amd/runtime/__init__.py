"""Native serving runtime (C++ via pybind11): block manager + batch builder, and the
shared-memory step channel used by tensor-parallel ranks.

The extension is built in-tree by ``ops/build.py``; importing this package builds it on
first use if the shared object is missing.
"""
from __future__ import annotations

import importlib
import os


def _load():
    try:
        return importlib.import_module("._atta_runtime", __name__)
    except ImportError:
        if os.environ.get("ATTA_NO_BUILD", "0") == "1":
            raise
        from ..ops.build import build_runtime

        build_runtime()
        return importlib.import_module("._atta_runtime", __name__)


_rt = _load()
BlockManager = _rt.BlockManager
ShmChannel = _rt.ShmChannel

__all__ = ["BlockManager", "ShmChannel"]
