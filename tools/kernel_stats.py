"""Per-kernel launch durations from a rocprofv3 --kernel-trace CSV, counting only the
full-size dispatches (the largest grid seen for that kernel), so that the small launches
of bench.py's parity-check engines do not dilute the mean.

usage: python tools/kernel_stats.py KERNEL_TRACE_CSV [--out JSON]"""
import argparse
import csv
import json
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = defaultdict(list)
    for r in csv.DictReader(open(a.trace)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if not name.startswith("k_"):
            continue
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        rows[name].append((grid, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6))
    out = {}
    for name, v in sorted(rows.items()):
        gmax = max(g for g, _ in v)
        full = [ms for g, ms in v if g == gmax]
        out[name] = {"grid": gmax, "launches": len(full), "other_launches": len(v) - len(full),
                     "mean_ms": statistics.mean(full), "min_ms": min(full), "max_ms": max(full)}
        print(f"{name:24s} grid {gmax:8d}  n {len(full):3d} (+{len(v) - len(full)} smaller)  "
              f"mean {out[name]['mean_ms']:.3f} ms  min {out[name]['min_ms']:.3f}  max {out[name]['max_ms']:.3f}")
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
