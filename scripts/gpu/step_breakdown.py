"""Kernel-time breakdown of one cached-burst prefill step from a rocprofv3 kernel-trace CSV
directory: the contiguous run of dispatches around the first wide small-M GEMM launch of at
least ``--mt-min`` 16-row blocks (the 50-105-row bursts of the fan-out bench), from the embed
kernel before it to the first decode-step kernel after it (start-up warm-up launches, which
have no embed kernel before them, are skipped).  Prints, per kernel class, the
launches and summed GPU time, plus the span's idle time.

    python scripts/gpu/step_breakdown.py DIR [--mt-min 4] [--nth 0]
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

d = sys.argv[1]
mt_min = int(sys.argv[sys.argv.index("--mt-min") + 1]) if "--mt-min" in sys.argv else 4
nth = int(sys.argv[sys.argv.index("--nth") + 1]) if "--nth" in sys.argv else 0
raw = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            raw.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "?")))
raw.sort()


def wide_mt(name):
    # wide_kernel<T, WAVES, MT, ...>: mangled ...wide_kernelI<T>Li<W>ELi<MT>E...
    m = re.search(r"wide_kernelI\w+?Li(\d+)ELi(\d+)E", name)
    return int(m.group(2)) if m else 0


def cls(name):
    for key in ("wide_reduce", "wide_kernel", "flash_prefill", "attention_decode", "decode_attention",
                "skinny_kernel", "embed_kernel", "rms_norm", "rope_cache", "sample", "Cijk",
                "copyBuffer"):
        if key in name:
            return key
    return name[:50]


starts = [i for i, r in enumerate(raw) if wide_mt(r[2]) >= mt_min]
if not starts:
    print("no wide launch with MT >=", mt_min)
    sys.exit(0)
# group wide launches into steps (a step's 32 layers are < 2 ms apart)
steps, cur = [], [starts[0]]
for i in starts[1:]:
    if raw[i][0] - raw[cur[-1]][1] > 2_000_000:
        steps.append(cur)
        cur = [i]
    else:
        cur.append(i)
steps.append(cur)


def embed_before(i):
    while i > 0 and "embed_kernel" not in raw[i][2]:
        i -= 1
    return i


# engine start-up warm-up launches (ops.warm_wide_kernels, EngineConfig.startup_warmup) have no
# embed kernel right before them: only groups within 2 ms of an embed launch are prefill steps
steps = [g for g in steps if raw[g[0]][0] - raw[embed_before(g[0])][1] < 2_000_000]
if not steps:
    print("no prefill step with a wide launch of MT >=", mt_min)
    sys.exit(0)
sel = steps[min(nth, len(steps) - 1)]
lo = embed_before(sel[0])
hi = sel[-1]
while hi + 1 < len(raw) and cls(raw[hi + 1][2]) not in ("skinny_kernel", "embed_kernel") and \
        raw[hi + 1][0] - raw[hi][1] < 1_000_000:
    hi += 1
span = raw[lo:hi + 1]
tot = defaultdict(float)
cnt = defaultdict(int)
for s, e, n in span:
    k = cls(n)
    if k == "wide_kernel":
        k = f"wide_kernel MT{wide_mt(n)}"
    tot[k] += (e - s) / 1e3
    cnt[k] += 1
wall = (span[-1][1] - span[0][0]) / 1e3
busy = sum(tot.values())
print(f"burst step {nth} of {len(steps)}: {len(span)} dispatches, wall {wall:.1f} us, "
      f"kernels {busy:.1f} us, idle {wall - busy:.1f} us")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {k:28s} {cnt[k]:5d} launches {v:9.1f} us  ({v / cnt[k]:6.1f} us each)")
