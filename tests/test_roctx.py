"""ROCTx ranges: no-ops by default, real roctx calls when ATTA_ROCTX=1 (library present)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_roctx_default_noop():
    from agentic_traffic_testing_amd.utils import roctx

    assert not roctx.ENABLED or os.environ.get("ATTA_ROCTX") == "1"
    with roctx.range("x"):
        pass
    roctx.mark("y")


def test_roctx_enabled_calls_library():
    code = ("from agentic_traffic_testing_amd.utils import roctx\n"
            "assert roctx.ENABLED\n"
            "with roctx.range('engine.step'):\n"
            "    roctx.mark('inside')\n"
            "print('lib', roctx._lib is not None)\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT,
                       env=dict(os.environ, ATTA_ROCTX="1", PYTHONPATH=ROOT), timeout=120)
    assert r.returncode == 0, r.stderr
    # the ROCm image ships rocprofiler-sdk's ROCTx library; elsewhere the calls stay no-ops
    if os.path.exists("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1"):
        assert "lib True" in r.stdout
