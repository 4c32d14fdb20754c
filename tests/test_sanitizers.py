"""Host-code sanitizer tier: the C++ runtime (paged-KV block manager, batch
builder, TP step channel) rebuilt with ASan + UBSan and driven by a randomized stress script
(scripts/sanitize_runtime.py) in a child process that preloads libasan.  GPU code is never
sanitized (no GPU ASan on this pool)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _libasan():
    r = subprocess.run(["g++", "-print-file-name=libasan.so"], capture_output=True, text=True)
    p = r.stdout.strip()
    return p if p and os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.skipif(_libasan() is None, reason="no libasan in this toolchain")
def test_runtime_under_asan_ubsan():
    from agentic_traffic_testing_amd.ops.build import build_runtime_sanitized

    so = build_runtime_sanitized()
    # libstdc++ preloaded next to libasan: python itself does not link it, and ASan's
    # __cxa_throw interceptor must resolve the real symbol at start-up
    stdcxx = subprocess.run(["g++", "-print-file-name=libstdc++.so"], capture_output=True,
                            text=True).stdout.strip()
    env = dict(os.environ, LD_PRELOAD=f"{_libasan()} {os.path.realpath(stdcxx)}",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "sanitize_runtime.py"),
                        str(so)], capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert r.returncode == 0 and "SANITIZED RUNTIME OK" in r.stdout, out[-4000:]
