"""Summarise a rocprofv3 kernel-trace CSV directory: top kernels by total time, plus
per-decode-step breakdown estimate."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
if not files:
    print("no kernel trace found"); sys.exit(0)
tot = defaultdict(float); cnt = defaultdict(int)
rows = []
for f in files:
    with open(f) as fh:
        for r in csv.DictReader(fh):
            name = r.get("Kernel_Name", "?")
            dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            tot[name] += dt; cnt[name] += 1
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
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
