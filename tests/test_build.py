"""The in-tree native libraries build for gfx950 and load on a CPU-only host (catches
undefined symbols / missing registrations before a GPU box ever sees them)."""
import torch

from agentic_traffic_testing_amd.ops import build

EXPECTED_OPS = {
    "rms_norm", "fused_add_rms_norm", "silu_and_mul", "embed", "stream_read", "rope_cache",
    "attention_prefill",
    "attention_decode", "attention_decode_v2", "sample", "skinny_gemm", "fused_qkv_rope",
    "fused_gate_up_silu", "fused_lm_head_sample", "sample_finalize", "skinny_variant",
    "ar_buffer_bytes", "ar_alloc", "ar_free", "ar_handle", "ar_open", "ar_close", "ar_error",
    "ar_run",
}


def test_kernel_library_loads_and_registers_all_ops():
    so = build.build_kernels()
    torch.ops.load_library(str(so))
    for name in EXPECTED_OPS:
        assert hasattr(torch.ops.atta, name), name
        getattr(torch.ops.atta, name).default  # schema registered
    # host-only helper callable without a GPU
    assert torch.ops.atta.ar_buffer_bytes(1024, 2) == 64 * 1024 + 2 * 8 * 1024 * 2


def test_runtime_extension_loads():
    from agentic_traffic_testing_amd.runtime import BlockManager, ShmChannel

    bm = BlockManager(8, 16, True)
    assert bm.num_free_blocks() == 8
    assert ShmChannel is not None


def test_embed_cpu_fallback_honours_lookahead_flag():
    from agentic_traffic_testing_amd import ops

    table = torch.randn(50, 16)
    ids = torch.tensor([1, 2, 3], dtype=torch.int32)
    prev = torch.tensor([7, 8, 9, 10], dtype=torch.int64)
    assert torch.equal(ops.embed(table, ids), table[[1, 2, 3]])
    assert torch.equal(ops.embed(table, ids, prev, torch.zeros(1, dtype=torch.int32)),
                       table[[1, 2, 3]])
    assert torch.equal(ops.embed(table, ids, prev, torch.ones(1, dtype=torch.int32)),
                       table[[7, 8, 9]])


def test_build_is_content_hashed(tmp_path, monkeypatch):
    """Staleness is decided by source CONTENT: the built library embeds the hash of the
    sources it came from, and any source edit changes the hash the loader expects."""
    import shutil

    from agentic_traffic_testing_amd import ops

    build.build_kernels()
    assert ops.library_build_hash() == build.kernel_source_hash()
    copy = tmp_path / "csrc"
    shutil.copytree(build.CSRC, copy)
    before = build.kernel_source_hash()
    monkeypatch.setattr(build, "CSRC", copy)
    assert build.kernel_source_hash() == before  # same bytes, other place/mtime
    (copy / "common.h").write_text((copy / "common.h").read_text() + "\n// edit\n")
    assert build.kernel_source_hash() != before


def test_runtime_embeds_source_hash():
    from agentic_traffic_testing_amd import runtime

    assert runtime.BUILD_HASH == build.runtime_source_hash()


def test_current_library_is_used_without_object_files(tmp_path, monkeypatch):
    """A gpurun snapshot ships the .so but not _build/*.o: a library that embeds the current
    source hash must load as is (no rebuild - N DP ranks import at once), and a stale one is
    detected from its bytes."""
    from agentic_traffic_testing_amd import ops

    build.build_kernels()
    assert ops._lib_embeds(build.kernel_source_hash())
    assert not ops._lib_embeds("0" * 32)
    calls = []
    monkeypatch.setattr(build, "build_kernels", lambda *a, **k: calls.append(1))
    monkeypatch.setattr(ops, "_loaded", False)
    assert ops.load_native(build_if_missing=True), ops._load_error
    assert calls == []


def test_build_lock_serialises_processes(tmp_path):
    """Two processes holding the build lock never overlap."""
    import subprocess
    import sys

    log = tmp_path / "log"
    code = (
        "import time, sys\n"
        "from agentic_traffic_testing_amd.ops import build\n"
        "with build._build_lock():\n"
        f"    open({str(log)!r}, 'a').write('in\\n'); time.sleep(0.5)\n"
        f"    open({str(log)!r}, 'a').write('out\\n')\n")
    ps = [subprocess.Popen([sys.executable, "-c", code]) for _ in range(2)]
    assert all(p.wait(timeout=60) == 0 for p in ps)
    assert log.read_text().split() == ["in", "out", "in", "out"]
