#!/usr/bin/env python3
"""Summarise the nodes of captured decode-step hipGraphs (``ATTA_GRAPH_DUMP_DIR`` dumps).

``ModelRunner.capture`` writes one ``.nodes`` file per captured (rank, bucket, partitions)
graph when ``ATTA_GRAPH_DUMP_DIR`` is set: the graph's node list read back with
hipGraphGetNodes / hipGraphKernelNodeGetParams (ops graph_nodes binding).  This lists, per
file, the node kinds (kernel / memcpy / memset / host / event ...) and the kernel names with
their counts, and flags collective kernels: the atta IPC kernels (``oneshot_kernel`` sums,
``keymax_kernel`` sampler MAX) vs RCCL (``nccl``/``rccl``) - the evidence that a TP decode
step is device-side end to end.

    python scripts/gpu/graph_nodes.py gpurun_out/graphs > profiles/r3_tp8_graph_nodes.txt
"""
from __future__ import annotations

import collections
import re
import shutil
import subprocess
import sys
from pathlib import Path


def demangle(names: list[str]) -> dict[str, str]:
    tool = shutil.which("llvm-cxxfilt") or "/opt/rocm/lib/llvm/bin/llvm-cxxfilt"
    try:
        out = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True,
                             timeout=30).stdout.splitlines()
        return dict(zip(names, out))
    except Exception:
        return {n: n for n in names}


def short(name: str) -> str:
    base = re.sub(r"\(.*$", "", name)          # drop the argument list
    base = re.sub(r"<.*>", "<..>", base)       # collapse template arguments
    return base.split("::")[-1] if "::" in base else base


def summarise(path: Path) -> str:
    lines = [x for x in path.read_text(errors="replace").splitlines() if x.strip()]
    kinds = collections.Counter(x.split(":", 1)[0] for x in lines)
    names = [x.split(":", 1)[1].split(" grid=")[0] for x in lines if x.startswith("kernel:")]
    dm = demangle(sorted({n for n in names if n.startswith("_Z")}))
    kern = collections.Counter(short(dm.get(n, n)) for n in names)
    lines = [f"== {path.name}: node kinds {dict(kinds)}"]
    for k, c in kern.most_common():
        tag = ""
        if ("oneshot_kernel" in k or "twoshot_kernel" in k or "keymax_kernel" in k
                or "push_reduce_kernel" in k):
            tag = "   <- IPC collective"
        elif re.search(r"nccl|rccl", k, re.I):
            tag = "   <- RCCL"
        lines.append(f"  {c:5d}  {k}{tag}")
    rccl = sum(c for k, c in kern.items() if re.search(r"nccl|rccl", k, re.I))
    ipc = sum(c for k, c in kern.items() if re.search(r"oneshot|twoshot|keymax|push_reduce", k))
    lines.append(f"  -> IPC collective kernels {ipc}, RCCL kernels {rccl}, host nodes "
                 f"{kinds.get('host', 0)}")
    return "\n".join(lines)


def main(argv: list[str]) -> int:
    root = Path(argv[1] if len(argv) > 1 else "gpurun_out/graphs")
    files = sorted(root.glob("*.nodes"))
    if not files:
        print(f"no .nodes files under {root}")
        return 1
    for f in files:
        print(summarise(f))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
