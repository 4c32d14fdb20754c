"""Run MCP-Universe benchmark domains against the testbed (reference
scripts/experiment/run_mcp_universe.py:1-166).

``MCP_UNIVERSE_DIR`` (or ``--mcp-universe-dir``) points at a checkout; domains are the
``tests/benchmark/mcpuniverse/test_benchmark_<domain>.py`` files found there (falling back
to the known list when discovery finds none).  Each domain runs as its own subprocess with
the checkout prepended to ``PYTHONPATH`` and cwd = checkout, so ``OPENAI_BASE_URL`` /
``OPENAI_API_KEY`` in the environment route it through ``tools.mcp_universe.openai_proxy``.

Exit codes: 1 when the checkout is missing, an unknown domain is named or any domain fails;
0 otherwise (``--list`` / no arguments included).
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
from pathlib import Path

BENCH_SUBDIR = Path("tests") / "benchmark" / "mcpuniverse"
KNOWN_DOMAINS = ("dummy", "location_navigation", "browser_automation", "financial_analysis",
                 "repository_management", "web_search", "3d_design")


def checkout_dir(arg: str | None) -> Path | None:
    raw = arg or os.environ.get("MCP_UNIVERSE_DIR", "")
    if not raw:
        return None
    p = Path(raw).resolve()
    return p if p.is_dir() else None


def discover(root: Path) -> dict[str, Path]:
    bench = root / BENCH_SUBDIR
    found = {f.stem[len("test_benchmark_"):]: f
             for f in sorted(bench.glob("test_benchmark_*.py"))} if bench.is_dir() else {}
    if not found:
        for name in KNOWN_DOMAINS:
            f = bench / f"test_benchmark_{name}.py"
            if f.exists():
                found[name] = f
    return found


def run_domains(root: Path, domains: list[str], benches: dict[str, Path]) -> list[str]:
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join(p for p in (str(root), env.get("PYTHONPATH")) if p)
    failed = []
    for d in domains:
        f = benches.get(d)
        if f is None or not f.exists():
            print(f"[SKIP] {d}: test file not found")
            continue
        print(f"\n[*] Running MCP-Universe benchmark: {d}", flush=True)
        if subprocess.run([sys.executable, str(f)], cwd=str(root), env=env).returncode != 0:
            failed.append(d)
    return failed


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description="Run MCP-Universe benchmarks from the testbed")
    ap.add_argument("domain", nargs="?", help="benchmark domain, e.g. dummy")
    ap.add_argument("--all", action="store_true", help="run every discovered domain")
    ap.add_argument("--list", action="store_true", help="list domains and exit")
    ap.add_argument("--mcp-universe-dir", default=None)
    a = ap.parse_args(argv)
    root = checkout_dir(a.mcp_universe_dir)
    if root is None:
        print("[ERROR] MCP-Universe directory not found. Set MCP_UNIVERSE_DIR or pass "
              "--mcp-universe-dir.", file=sys.stderr)
        print("  Example: export MCP_UNIVERSE_DIR=/path/to/MCP-Universe", file=sys.stderr)
        return 1
    benches = discover(root)
    if a.list:
        print("Available MCP-Universe benchmark domains:")
        for name in sorted(benches):
            print(f"  {name}")
        return 0
    if a.all:
        domains = sorted(benches)
    elif a.domain:
        if a.domain not in benches:
            print(f"[ERROR] Unknown domain: {a.domain}", file=sys.stderr)
            print(f"  Available: {', '.join(sorted(benches))}", file=sys.stderr)
            return 1
        domains = [a.domain]
    else:
        ap.print_help()
        return 0
    failed = run_domains(root, domains, benches)
    if failed:
        print(f"\n[FAILED] {len(failed)} benchmark(s): {', '.join(failed)}", file=sys.stderr)
        return 1
    print("\n[OK] All benchmarks completed successfully.")
    return 0


if __name__ == "__main__":
    sys.exit(main())
