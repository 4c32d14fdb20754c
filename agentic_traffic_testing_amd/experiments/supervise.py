"""Supervised long experiment (reference scripts/experiment/run_aggregated_experiment.sh and
monitor_experiment.sh, SURVEY §2.2 E5 / §5.3 recovery).

The reference starts the runner under nohup, installs a ``*/5`` cron job and lets the cron
check restart a crashed runner in resume mode.  Here one supervisor process owns the
runner as a child:

* ``supervise(...)`` waits ``settle_s`` (default 300 s, "let metrics pipelines settle"),
  starts ``runner -n N -o DIR``, and whenever the child exits without ``DONE`` in
  ``summary.txt`` - or makes no progress (summary.txt unchanged) for ``stall_s`` - it is
  stopped (exact PID) and restarted with ``-c -o DIR``, up to ``max_restarts`` times;
* the state file (JSON: pid, experiment_dir) is kept for ``check`` - a one-shot probe for
  cron-style use that restarts a dead, unfinished experiment exactly like the reference's
  monitor script (no crontab editing needed).
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
DEFAULT_STATE = REPO / "data" / ".experiment_state.json"


def runner_cmd(args: list[str]) -> list[str]:
    return [sys.executable, "-m", "agentic_traffic_testing_amd.experiments.runner", *args]


def is_done(exp_dir: Path) -> bool:
    s = exp_dir / "summary.txt"
    return s.exists() and "  DONE" in s.read_text(encoding="utf-8", errors="replace")


def alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except OSError:
        return False
    try:  # a zombie child still "exists"
        done, _ = os.waitpid(pid, os.WNOHANG)
        return done == 0
    except ChildProcessError:
        return True


def _start(args: list[str], log: Path) -> subprocess.Popen:
    log.parent.mkdir(parents=True, exist_ok=True)
    fh = open(log, "a")
    return subprocess.Popen(runner_cmd(args), stdout=fh, stderr=subprocess.STDOUT, cwd=str(REPO),
                            start_new_session=True)


def _write_state(state: Path, pid: int, exp_dir: Path):
    state.parent.mkdir(parents=True, exist_ok=True)
    state.write_text(json.dumps({"pid": pid, "experiment_dir": str(exp_dir)}))


def supervise(iterations: int, exp_dir: Path, extra: list[str] | None = None,
              settle_s: float = 300.0, stall_s: float = 3600.0, max_restarts: int = 20,
              poll_s: float = 10.0, state: Path = DEFAULT_STATE) -> int:
    extra = extra or []
    if settle_s > 0:
        print(f"[supervise] waiting {settle_s:.0f}s for services/metrics to settle", flush=True)
        time.sleep(settle_s)
    log = exp_dir / "supervisor.log"
    proc = _start(["-n", str(iterations), "-o", str(exp_dir), *extra], log)
    restarts = 0
    while True:
        _write_state(state, proc.pid, exp_dir)
        last_size, last_change = -1, time.time()
        while proc.poll() is None:
            time.sleep(poll_s)
            s = exp_dir / "summary.txt"
            size = s.stat().st_size if s.exists() else 0
            if size != last_size:
                last_size, last_change = size, time.time()
            elif time.time() - last_change > stall_s:
                print(f"[supervise] no progress for {stall_s:.0f}s; stopping pid {proc.pid}",
                      flush=True)
                proc.send_signal(signal.SIGTERM)
                try:
                    proc.wait(30)
                except subprocess.TimeoutExpired:
                    proc.kill()
                    proc.wait()
        if is_done(exp_dir):
            print("[supervise] experiment completed", flush=True)
            if state.exists():
                state.unlink()
            return 0
        if restarts >= max_restarts:
            print("[supervise] giving up after too many restarts", flush=True)
            return 1
        restarts += 1
        print(f"[supervise] runner exited (rc={proc.returncode}) without DONE; "
              f"restart {restarts}/{max_restarts} in resume mode", flush=True)
        proc = _start(["-c", "-o", str(exp_dir), *extra], log)


def check(state: Path = DEFAULT_STATE) -> int:
    """One-shot monitor (cron): restart a dead, unfinished experiment in resume mode."""
    print(f"[monitor] {time.strftime('%Y-%m-%d %H:%M:%S')}")
    if not state.exists():
        print("[monitor] No state file found")
        return 0
    st = json.loads(state.read_text())
    exp_dir, pid = Path(st["experiment_dir"]), int(st["pid"])
    if alive(pid):
        print(f"[monitor] pid {pid} still running")
        return 0
    if is_done(exp_dir):
        print("[monitor] Experiment completed normally")
        state.unlink()
        return 0
    print("[monitor] Experiment appears to have crashed; restarting in resume mode")
    proc = _start(["-c", "-o", str(exp_dir)], exp_dir / "restart.log")
    _write_state(state, proc.pid, exp_dir)
    return 0


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description="Supervised experiment run with auto-resume")
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("-n", type=int, required=True)
    r.add_argument("-o", default=None)
    r.add_argument("--settle-s", type=float, default=300.0)
    r.add_argument("--stall-s", type=float, default=3600.0)
    r.add_argument("--max-restarts", type=int, default=20)
    r.add_argument("--state", default=str(DEFAULT_STATE))
    r.add_argument("extra", nargs=argparse.REMAINDER, help="extra runner args after --")
    c = sub.add_parser("check")
    c.add_argument("--state", default=str(DEFAULT_STATE))
    a = ap.parse_args(argv)
    if a.cmd == "check":
        return check(Path(a.state))
    exp = Path(a.o) if a.o else REPO / "data" / "runs" / (
        "experiment_" + time.strftime("%Y-%m-%d_%H-%M-%S"))
    extra = [x for x in a.extra if x != "--"]
    return supervise(a.n, exp, extra, a.settle_s, a.stall_s, a.max_restarts, state=Path(a.state))


if __name__ == "__main__":
    sys.exit(main())
