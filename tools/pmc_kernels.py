"""Per-kernel PMC summary: for every render kernel, counters of its last dispatch, per wave
and per 128-sample block.  usage: python tools/pmc_kernels.py BLOCKS DIR [DIR ...]"""
import csv
import sys
from collections import defaultdict
from pathlib import Path


def main():
    blocks = int(sys.argv[1])
    agg = defaultdict(lambda: defaultdict(float))
    for d in sys.argv[2:]:
        f = next(Path(d).rglob("*counter_collection.csv"))
        last = {}
        rows = list(csv.DictReader(open(f)))
        for r in rows:
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            last[k] = max(last.get(k, -1), int(r["Dispatch_Id"]))
        for r in rows:
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if int(r["Dispatch_Id"]) == last[k] and k.startswith("k_"):
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, c in agg.items():
        w = c.get("SQ_WAVES", 1)
        print(f"== {k}  waves {w:.0f}")
        for n in sorted(c):
            print(f"   {n:28s} {c[n]:14.4g}  per wave-block {c[n] / w / blocks:12.1f}")


if __name__ == "__main__":
    main()
