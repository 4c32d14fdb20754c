"""Print the kernel sequence of a rocprofv3 kernel-trace CSV between two dispatch indices
(default: the 60 dispatches before the last occurrence of a marker kernel)."""
import csv
import glob
import os
import sys

d = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "sample"
n = int(sys.argv[3]) if len(sys.argv) > 3 else 60
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
last = max((i for i, r in enumerate(rows) if marker in r[2]), default=len(rows) - 1)
for s, e, name in rows[max(0, last - n):last + 1]:
    print(f"{(e - s) / 1e3:9.2f} us  {name[:120]}")
