"""HBM bytes per launch of each render kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE passes
over bench.py, corrected as calibrated on MI355X (profiles/r01_pmc_calibration.txt:
FETCH_SIZE x 2 and WRITE_SIZE x 1 for the kernels' 8-B/lane streams).

usage: python tools/traffic_from_pmc.py FETCH_DIR WRITE_DIR --batch 4096 --blocks 64 \
           --sr 48000 --chain 0 --out profiles/traffic.json
bench.py reports roofline.traffic from the output when its workload matches."""
import argparse
import csv
import json
import statistics
from collections import defaultdict
from pathlib import Path

FETCH_SCALE, WRITE_SCALE = 2.0, 1.0
KERNELS = ("k_tonegen", "k_mixpre", "k_rv_pre", "k_rv_core", "k_rv_post", "k_whirl")


def per_dispatch(d, counter):
    f = next(Path(d).rglob("*counter_collection.csv"))
    agg = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        k = int(r["Dispatch_Id"])
        agg[k] += float(r["Counter_Value"])
        names[k] = r["Kernel_Name"]
    out = defaultdict(list)
    for k, v in agg.items():
        for kn in KERNELS:
            if kn in names[k]:
                out[kn].append(v * 1024.0)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--blocks", type=int, default=64)
    ap.add_argument("--sr", type=float, default=48000.0)
    ap.add_argument("--chain", type=int, default=0)
    ap.add_argument("--out", default="profiles/traffic.json")
    a = ap.parse_args()
    fe, wr = per_dispatch(a.fetch_dir, "FETCH_SIZE"), per_dispatch(a.write_dir, "WRITE_SIZE")
    samples = a.batch * a.blocks * 128
    res = {"workload": {"batch": a.batch, "blocks": a.blocks, "sr": a.sr, "chain": a.chain},
           "fetch_scale": FETCH_SCALE, "write_scale": WRITE_SCALE,
           "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes: {a.fetch_dir}, {a.write_dir}",
           "kernels": {}}
    for k in KERNELS:
        if k not in fe or k not in wr:
            continue
        # the workload's full launches only (bench.py also renders small check / stage-tap
        # runs): the median over the dispatches within half of the largest
        full = lambda v: [x for x in v if x >= 0.5 * max(v)]
        rb = statistics.median(full(fe[k])) * FETCH_SCALE
        wb = statistics.median(full(wr[k])) * WRITE_SCALE
        res["kernels"][k] = {"read_bytes": rb, "write_bytes": wb, "bytes_per_launch": rb + wb,
                             "bytes_per_stereo_sample": (rb + wb) / samples, "launches": len(full(fe[k]))}
    Path(a.out).write_text(json.dumps(res, indent=1))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
