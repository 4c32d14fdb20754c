"""Native serving runtime (C++ via pybind11): block manager + batch builder, and the
shared-memory step channel used by tensor-parallel ranks.

The extension is built in-tree by ``ops/build.py`` (content-hash stamped); importing this
package (re)builds it when its sources changed, unless ``ATTA_NO_BUILD=1``, in which case
a binary whose embedded ``BUILD_HASH`` does not match the sources is refused.
"""
from __future__ import annotations

import importlib
import os


class StaleNativeBuild(ImportError):
    pass


def _load():
    from ..ops import build

    if os.environ.get("ATTA_NO_BUILD", "0") != "1":
        build.build_runtime()  # no-op when the stamp matches the sources
    mod = importlib.import_module("._atta_runtime", __name__)
    want = build.runtime_source_hash()
    if getattr(mod, "BUILD_HASH", None) != want:
        raise StaleNativeBuild(
            f"_atta_runtime was built from other sources (BUILD_HASH "
            f"{getattr(mod, 'BUILD_HASH', None)} != {want}); run "
            "`python -m agentic_traffic_testing_amd.ops.build`")
    return mod


_rt = _load()
BlockManager = _rt.BlockManager
ShmChannel = _rt.ShmChannel
BUILD_HASH = _rt.BUILD_HASH

__all__ = ["BlockManager", "ShmChannel", "BUILD_HASH", "StaleNativeBuild"]
