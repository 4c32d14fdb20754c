"""Summarise a rocprofv3 kernel-trace CSV directory: top kernels by total time, plus
per-decode-step breakdown estimate."""
import csv
import glob
import os
import sys
from collections import defaultdict

# usage: summarize_trace.py DIR [--window MARKER]
# --window: only the dispatches strictly between the first and the last dispatch of a kernel
# whose name contains MARKER (e.g. stream_read_kernel, which scripts/gpu/prefill_bench.py
# launches around its measured region): model init and warm-up stay out of the table.
d = sys.argv[1]
window = sys.argv[sys.argv.index("--window") + 1] if "--window" in sys.argv else None
files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
if not files:
    print("no kernel trace found"); sys.exit(0)
raw = []
for f in files:
    with open(f) as fh:
        for r in csv.DictReader(fh):
            raw.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                        r.get("Kernel_Name", "?")))
raw.sort()
if window:
    idx = [i for i, r in enumerate(raw) if window in r[2]]
    if len(idx) >= 2:
        raw = raw[idx[0] + 1:idx[-1]]
        raw = [r for r in raw if window not in r[2]]
        print(f"window: dispatches between the first and last {window} ({len(raw)} kernels)")
    else:
        print(f"window marker {window} not found twice: whole trace")
tot = defaultdict(float); cnt = defaultdict(int)
rows = []
for s_, e_, name in raw:
    dt = (e_ - s_) / 1e3
    tot[name] += dt; cnt[name] += 1
    rows.append((s_, e_, name))
all_t = sum(tot.values())
print(f"kernels: {sum(cnt.values())} dispatches, {all_t/1e3:.1f} ms total GPU time")
print(f"{'total_ms':>10} {'calls':>8} {'avg_us':>9} {'pct':>6}  kernel")
for name, t in sorted(tot.items(), key=lambda x: -x[1])[:40]:
    short = name if len(name) < 110 else name[:107] + "..."
    print(f"{t/1e3:10.2f} {cnt[name]:8d} {t/cnt[name]:9.2f} {100*t/all_t:6.2f}  {short}")
rows.sort()
if rows:
    span = (rows[-1][1] - rows[0][0]) / 1e6
    print(f"\nwall span of traced kernels: {span:.1f} ms; busy {all_t/1e3:.1f} ms ({100*all_t/1e3/span:.1f}%)")

# Gaps between back-to-back kernels of the decode step (graph replay): for every pair of
# consecutive dispatches where both are atta decode kernels, start[i+1] - end[i].
def short_name(n):
    for key in ("skinny_kernel", "decode_attention_kernel", "sample_finalize", "oneshot"):
        if key in n:
            return key
    return None


gaps = defaultdict(list)
for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
    a, b = short_name(n0), short_name(n1)
    if a and b and 0 <= s1 - e0 < 100_000:  # same step (< 100 us apart)
        gaps[f"{a} -> {b}"].append((s1 - e0) / 1e3)
if gaps:
    import statistics
    print("\ninter-kernel gaps inside decode steps (us): pair, count, median, p90")
    for k, v in sorted(gaps.items(), key=lambda kv: -len(kv[1])):
        v.sort()
        print(f"  {k:50s} {len(v):7d} {statistics.median(v):7.2f} {v[int(0.9 * (len(v) - 1))]:7.2f}")

# Where the GPU idles: every gap between consecutive dispatches (any kernels), by size bucket,
# and the kernel pairs that hold the most idle time in total.
def pair_name(n):
    k = short_name(n)
    if k:
        return k
    for key in ("embed_kernel", "wide_kernel", "wide_reduce", "flash_prefill", "rms_norm",
                "rope_cache", "Cijk", "copyBuffer", "fillBuffer", "stream_read"):
        if key in n:
            return key
    return n[:40]


if len(rows) > 1:
    buckets = [(5, "<5us"), (20, "5-20us"), (100, "20-100us"), (1000, "0.1-1ms"),
               (float("inf"), ">1ms")]
    bsum = defaultdict(float); bcnt = defaultdict(int)
    psum = defaultdict(float); pcnt = defaultdict(int)
    for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
        g = (s1 - e0) / 1e3
        if g <= 0:
            continue
        lab = next(lab for lim, lab in buckets if g < lim)
        bsum[lab] += g; bcnt[lab] += 1
        key = f"{pair_name(n0)} -> {pair_name(n1)}"
        psum[key] += g; pcnt[key] += 1
    print("\nidle gaps between consecutive dispatches: bucket, count, total ms")
    for _, lab in buckets:
        print(f"  {lab:10s} {bcnt[lab]:8d} {bsum[lab] / 1e3:9.2f}")
    print("kernel pairs holding the most idle time: pair, count, total ms, mean us")
    for k, v in sorted(psum.items(), key=lambda kv: -kv[1])[:15]:
        print(f"  {k:60s} {pcnt[k]:7d} {v / 1e3:8.2f} {v / pcnt[k]:8.1f}")
