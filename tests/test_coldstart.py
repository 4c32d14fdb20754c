"""Engine start warms every code object the serving paths reach.

HIP loads a translation unit's code object at the first launch of one of its kernels and
rocBLAS / hipBLASLt load a solution's at its first use; without the engine's start-up warm-up
(EngineConfig.startup_warmup: ops.warm_wide_kernels, ModelRunner.warm_library_gemms, throw-away
requests of the workload's step shapes in LLMEngine.warmup) the first request of a shape paid
it: 17-row planning 154 ms vs 3.7, 560-row prefill 1157 ms vs 11.5, 475-row burst 11.4 vs 9.3
(bench/coldstart.py on MI355X, round 6).  Here a FRESH process (nothing loaded by earlier
tests) builds bench.py's llama-3.1-8b engine and serves every fan-out step shape twice: the
first-ever occurrence must be within 10 % (+ 0.3 ms of host jitter) of the second."""
import json
import os
import subprocess
import sys

import pytest


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_first_request_of_every_step_shape_is_warm():
    env = dict(os.environ, ATTA_NO_BUILD="1")
    r = subprocess.run([sys.executable, "-u", "-m", "agentic_traffic_testing_amd.bench.coldstart",
                        "--reps", "2"], env=env, capture_output=True, text=True, timeout=800)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])["ttft_ms"]
    print(res)
    bad = {s: v for s, v in res.items() if v[0] > 1.10 * v[1] + 0.3}
    assert not bad, f"first occurrence slower than the repeat (ms): {bad}"
