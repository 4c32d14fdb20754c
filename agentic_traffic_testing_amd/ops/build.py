"""In-tree build of the native libraries (gfx950 HIP kernels + C++ runtime).

Produces, next to the sources (so the .so files travel with a gpurun snapshot):

* ``ops/_atta_kernels.so``  - CDNA4 HIP kernels + torch operator registration
  (``torch.ops.atta.*``), compiled with ``hipcc --offload-arch=gfx950``.
* ``runtime/_atta_runtime*.so`` - C++ block manager / batch builder (pybind11, g++).

No torch.utils.cpp_extension / hipify: sources are plain HIP written for CDNA4 and are
compiled with explicit hipcc command lines.  Builds are incremental (mtime based) and
parallel.

Usage:  python -m agentic_traffic_testing_amd.ops.build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent.parent
OPS = PKG / "ops"
CSRC = OPS / "csrc"
BUILD = OPS / "_build"
KERNEL_SO = OPS / "_atta_kernels.so"
RUNTIME_DIR = PKG / "runtime"
RUNTIME_CSRC = RUNTIME_DIR / "csrc"

ARCH = os.environ.get("ATTA_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")


def _torch_paths():
    import torch  # noqa: F401
    from torch.utils import cpp_extension as ce

    return ce.include_paths(), ce.library_paths()


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return r


def build_kernels(force: bool = False, jobs: int = 8, verbose: bool = False) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    headers = list(CSRC.glob("*.h"))
    hip_srcs = sorted(CSRC.glob("*.hip"))
    objs = []
    cmds = []
    for src in hip_srcs:
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        if force or _stale(obj, [src, *headers]):
            cmds.append([
                HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                "-munsafe-fp-atomics", "-Wno-unused-result", "-I", str(CSRC),
                "-c", str(src), "-o", str(obj),
            ])
    inc, libdirs = _torch_paths()
    bind_src = CSRC / "bindings.cpp"
    bind_obj = BUILD / "bindings.o"
    objs.append(bind_obj)
    if force or _stale(bind_obj, [bind_src, *headers]):
        cmd = [HIPCC, "-O2", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__=1",
               "-DUSE_ROCM=1", "-D_GLIBCXX_USE_CXX11_ABI=1", "-Wno-unused-result",
               "-Wno-deprecated-declarations", "-I", str(CSRC)]
        for i in inc:
            cmd += ["-I", i]
        cmd += ["-c", str(bind_src), "-o", str(bind_obj)]
        cmds.append(cmd)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for r in ex.map(_run, cmds):
            if verbose and (r.stdout or r.stderr):
                print(r.stdout, r.stderr)
    if force or cmds or _stale(KERNEL_SO, objs):
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(KERNEL_SO), *map(str, objs)]
        for d in libdirs:
            link += ["-L", d, f"-Wl,-rpath,{d}"]
        link += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip"]
        _run(link)
    return KERNEL_SO


def runtime_so_path() -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return RUNTIME_DIR / f"_atta_runtime{suffix}"


def build_runtime(force: bool = False) -> Path:
    import pybind11

    target = runtime_so_path()
    srcs = sorted(RUNTIME_CSRC.glob("*.cpp"))
    hdrs = sorted(RUNTIME_CSRC.glob("*.h"))
    if not srcs:
        raise RuntimeError("no runtime sources")
    if force or _stale(target, [*srcs, *hdrs]):
        py_inc = sysconfig.get_paths()["include"]
        cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wno-unused-function",
               "-I", pybind11.get_include(), "-I", py_inc, "-I", str(RUNTIME_CSRC),
               *map(str, srcs), "-o", str(target)]
        _run(cmd)
    return target


def build_all(force: bool = False, jobs: int = 8, verbose: bool = False):
    rt = build_runtime(force=force)
    ks = build_kernels(force=force, jobs=jobs, verbose=verbose)
    return ks, rt


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args(argv)
    ks, rt = build_all(force=a.force, jobs=a.j, verbose=a.v)
    print(f"built {ks}\nbuilt {rt}")


if __name__ == "__main__":
    sys.exit(main())
