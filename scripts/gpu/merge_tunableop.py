"""Merge a TunableOp results CSV (e.g. a longer re-tune of some row buckets) into the shipped
table: an entry is replaced only when the new solution's measured time is lower by more than
--margin (the two tunings ran on different boxes, so small differences are noise).

    python scripts/gpu/merge_tunableop.py gpurun_out/tun_large.csv \
        agentic_traffic_testing_amd/tuning/tunableop_gfx950_llama-3.1-8b.csv --margin 0.05
"""
import argparse


def read(path):
    head, rows = [], {}
    with open(path) as f:
        for line in f:
            line = line.rstrip("\n")
            if not line:
                continue
            parts = line.split(",")
            if parts[0] == "Validator":
                head.append(line)
            elif len(parts) >= 4:
                rows[(parts[0], parts[1])] = (parts[2], float(parts[3]))
    return head, rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("new")
    ap.add_argument("table")
    ap.add_argument("--margin", type=float, default=0.05)
    ap.add_argument("--dry-run", action="store_true")
    a = ap.parse_args()
    head, old = read(a.table)
    _, new = read(a.new)
    out = dict(old)
    for key, (sol, t) in new.items():
        prev = old.get(key)
        if prev is None or t < prev[1] * (1.0 - a.margin):
            out[key] = (sol, t)
            was = f"{prev[0]} {prev[1] * 1e3:8.1f} us" if prev else "(absent)"
            print(f"{key[1]:45s} {was} -> {sol} {t * 1e3:8.1f} us")
    if not a.dry_run:
        with open(a.table, "w") as f:
            for line in head:
                f.write(line + "\n")
            for (op, shape), (sol, t) in out.items():
                f.write(f"{op},{shape},{sol},{t}\n")
    print(f"# {sum(1 for k in new if out[k] == new[k])} of {len(new)} entries taken")


if __name__ == "__main__":
    main()
