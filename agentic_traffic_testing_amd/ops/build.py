"""In-tree build of the native libraries (gfx950 HIP kernels + C++ runtime).

Produces, next to the sources (so the .so files travel with a gpurun snapshot):

* ``ops/_atta_kernels.so``  - CDNA4 HIP kernels + torch operator registration
  (``torch.ops.atta.*``), compiled with ``hipcc --offload-arch=gfx950``.
* ``runtime/_atta_runtime*.so`` - C++ block manager / batch builder / TP step channel
  (pybind11, g++).

No torch.utils.cpp_extension / hipify: sources are plain HIP written for CDNA4 and are
compiled with explicit hipcc command lines.

Staleness is decided by CONTENT, not mtimes: every object has a ``.stamp`` holding the
sha256 of its compile command plus the bytes of its source and of every header in its
directory, and each library embeds the hash of all its sources (``atta_build_hash()`` in
the kernel library, ``BUILD_HASH`` in the runtime module).  The loaders
(``ops.load_native`` / ``runtime._load``) compare that hash against the sources on disk
and refuse a stale library, so a snapshot whose sources moved on without a rebuild fails
loudly instead of running old kernels.

Usage:  python -m agentic_traffic_testing_amd.ops.build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import contextlib
import fcntl
import hashlib
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


def _sha(parts) -> str:
    h = hashlib.sha256()
    for p in parts:
        h.update(p if isinstance(p, bytes) else str(p).encode())
        h.update(b"\0")
    return h.hexdigest()


def _files_digest(files) -> list:
    out = []
    for f in sorted(Path(x) for x in files):
        out += [f.name, f.read_bytes()]
    return out


def kernel_sources() -> list[Path]:
    return sorted([*CSRC.glob("*.hip"), *CSRC.glob("*.h"), *CSRC.glob("*.cpp")])


def runtime_sources() -> list[Path]:
    return sorted([*RUNTIME_CSRC.glob("*.cpp"), *RUNTIME_CSRC.glob("*.h")])


def kernel_source_hash() -> str:
    """Hash of every kernel-library source (what ``atta_build_hash()`` must return)."""
    return _sha(["kernels", ARCH, *_files_digest(kernel_sources())])[:32]


def runtime_source_hash() -> str:
    return _sha(["runtime", *_files_digest(runtime_sources())])[:32]


def _stamp_ok(target: Path, digest: str) -> bool:
    st = target.with_name(target.name + ".stamp")
    return target.exists() and st.exists() and st.read_text().strip() == digest


def _write_stamp(target: Path, digest: str):
    target.with_name(target.name + ".stamp").write_text(digest + "\n")


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return r


@contextlib.contextmanager
def _build_lock():
    """Exclusive inter-process lock around a build: ranks that import the package at the
    same time build once, in turn, instead of writing the same objects concurrently."""
    BUILD.mkdir(parents=True, exist_ok=True)
    with open(BUILD / ".build.lock", "w") as f:
        fcntl.flock(f, fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(f, fcntl.LOCK_UN)


def build_kernels(force: bool = False, jobs: int = 8, verbose: bool = False) -> Path:
    with _build_lock():
        return _build_kernels(force, jobs, verbose)


def _build_kernels(force: bool, jobs: int, verbose: bool) -> Path:
    headers = sorted(CSRC.glob("*.h"))
    hdr_digest = _files_digest(headers)
    src_hash = kernel_source_hash()
    # the library's identity: generated translation unit returning the source hash
    info = BUILD / "build_info.cpp"
    info_src = (f'extern "C" const char* atta_build_hash() {{ return "{src_hash}"; }}\n')
    if not info.exists() or info.read_text() != info_src:
        info.write_text(info_src)
    jobs_ = []  # (cmd, obj, digest)
    objs = []
    for src in sorted(CSRC.glob("*.hip")):
        obj = BUILD / (src.stem + ".o")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
               "-munsafe-fp-atomics", "-Wno-unused-result", "-I", str(CSRC),
               "-c", str(src), "-o", str(obj)]
        objs.append(obj)
        jobs_.append((cmd, obj, _sha([*cmd, src.read_bytes(), *hdr_digest])))
    inc, libdirs = _torch_paths()
    bind_src = CSRC / "bindings.cpp"
    bind_obj = BUILD / "bindings.o"
    cmd = [HIPCC, "-O2", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__=1",
           "-DUSE_ROCM=1", "-D_GLIBCXX_USE_CXX11_ABI=1", "-Wno-unused-result",
           "-Wno-deprecated-declarations", "-I", str(CSRC)]
    for i in inc:
        cmd += ["-I", i]
    cmd += ["-c", str(bind_src), "-o", str(bind_obj)]
    objs.append(bind_obj)
    jobs_.append((cmd, bind_obj, _sha([*cmd, bind_src.read_bytes(), *hdr_digest])))
    info_obj = BUILD / "build_info.o"
    cmd = ["g++", "-O2", "-fPIC", "-c", str(info), "-o", str(info_obj)]
    objs.append(info_obj)
    jobs_.append((cmd, info_obj, _sha([*cmd, info_src])))
    todo = [j for j in jobs_ if force or not _stamp_ok(j[1], j[2])]

    def compile_one(j):
        cmd_, obj_, dig = j
        r = _run(cmd_)
        _write_stamp(obj_, dig)
        return r

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for r in ex.map(compile_one, todo):
            if verbose and (r.stdout or r.stderr):
                print(r.stdout, r.stderr)
    link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(KERNEL_SO),
            *map(str, objs)]
    for d in libdirs:
        link += ["-L", d, f"-Wl,-rpath,{d}"]
    link += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip"]
    link_digest = _sha([*link, *(j[2] for j in jobs_)])
    if force or todo or not _stamp_ok(KERNEL_SO, link_digest):
        _run(link)
        _write_stamp(KERNEL_SO, link_digest)
    return KERNEL_SO


def runtime_so_path() -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return RUNTIME_DIR / f"_atta_runtime{suffix}"


def runtime_flags(extra=()) -> list[str]:
    import pybind11

    py_inc = sysconfig.get_paths()["include"]
    return ["-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", *extra,
            "-I", pybind11.get_include(), "-I", py_inc, "-I", str(RUNTIME_CSRC),
            f'-DATTA_BUILD_HASH="{runtime_source_hash()}"']


def build_runtime(force: bool = False) -> Path:
    with _build_lock():
        return _build_runtime(force)


def _build_runtime(force: bool) -> Path:
    target = runtime_so_path()
    srcs = sorted(RUNTIME_CSRC.glob("*.cpp"))
    if not srcs:
        raise RuntimeError("no runtime sources")
    cmd = ["g++", "-O3", "-shared", *runtime_flags(), *map(str, srcs), "-o", str(target)]
    digest = _sha([*cmd, *_files_digest(runtime_sources())])
    if force or not _stamp_ok(target, digest):
        _run(cmd)
        _write_stamp(target, digest)
    return target


SANITIZE_FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                  "-fno-sanitize-recover=undefined"]


def sanitized_runtime_path() -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return RUNTIME_DIR / "_asan" / f"_atta_runtime{suffix}"


def build_runtime_sanitized(force: bool = False) -> Path:
    """ASan + UBSan build of the host runtime (block manager, step channel) for the CPU
    sanitizer tier: same sources, own directory, loaded only by
    tests/test_sanitizers.py under LD_PRELOAD=libasan (never by the serving stack)."""
    target = sanitized_runtime_path()
    target.parent.mkdir(parents=True, exist_ok=True)
    srcs = sorted(RUNTIME_CSRC.glob("*.cpp"))
    flags = [f for f in runtime_flags() if f != "-O3"]
    cmd = ["g++", "-shared", *SANITIZE_FLAGS, *flags, *map(str, srcs), "-o", str(target)]
    digest = _sha([*cmd, *_files_digest(runtime_sources())])
    if force or not _stamp_ok(target, digest):
        _run(cmd)
        _write_stamp(target, digest)
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
