"""Summarise rocprofv3 counter CSVs: per-wave-per-block counts for tbf_render_kernel.
usage: python tools/pmc_summary.py DIR [blocks_per_launch]"""
import csv
import sys
from collections import defaultdict
from pathlib import Path


def load(d):
    f = next(Path(d).rglob("*counter_collection.csv"))
    agg = defaultdict(float)
    disp = set()
    for r in csv.DictReader(open(f)):
        if "tbf_render" not in r["Kernel_Name"]:
            continue
        disp.add(r["Dispatch_Id"])
        agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    last = sorted(disp, key=int)[-1]
    return {k[1]: v for k, v in agg.items() if k[0] == last}


if __name__ == "__main__":
    blocks = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    c = load(sys.argv[1])
    w = c.get("SQ_WAVES", 1)
    for k in sorted(c):
        print(f"{k:24s} {c[k]:14.4g}  per wave-block {c[k] / w / blocks:10.1f}")
