"""Print the kernel sequence (name, us) of one transformer layer from a rocprofv3 kernel-trace
CSV directory, windowed like summarize_trace.py: which library GEMM serves which projection.

    python scripts/gpu/layer_sequence.py DIR --window stream_read_kernel [--skip 40] [--n 12]
"""
import csv
import glob
import os
import sys

d = sys.argv[1]
window = sys.argv[sys.argv.index("--window") + 1] if "--window" in sys.argv else None
skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 40
n = int(sys.argv[sys.argv.index("--n") + 1]) if "--n" in sys.argv else 12
raw = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            raw.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "?"),
                        r.get("Grid_Size", r.get("Grid_Size_X", "?")), r.get("Workgroup_Size", "?")))
raw.sort()
if window:
    idx = [i for i, r in enumerate(raw) if window in r[2]]
    if len(idx) >= 2:
        raw = [r for r in raw[idx[0] + 1:idx[-1]] if window not in r[2]]
for s_, e_, name, grid, wg in raw[skip:skip + n]:
    print(f"{(e_ - s_) / 1e3:9.2f} us  grid {grid:>8} wg {wg:>5}  {name[:110]}")
