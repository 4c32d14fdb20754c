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
