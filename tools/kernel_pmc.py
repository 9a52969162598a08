"""Per-kernel PMC profile of one build: HBM bytes and SQ instruction / cycle counters per
launch of each render stage, from separate rocprofv3 --pmc passes over the same bench
command (MI355X_MICROARCH.md, HBM/rocprofv3 section: FETCH_SIZE and WRITE_SIZE each in a
pass of their own; FETCH_SIZE x 2 and WRITE_SIZE x 1 as calibrated for these kernels'
streams in profiles/r01_pmc_calibration.txt).

bench.py reads the output (profiles/kernel_pmc.json) and divides the per-launch counts by
each kernel's unloaded launch time, measured live, to report every kernel against the
ceiling that binds it (HBM bytes, VALU issue) -- only when the build hash matches.

The counters are per launch, so per --launch-blocks blocks (the engine's steady chunk the
profiled bench rendered in; bench.py scales them to the launches it times).

usage: python tools/kernel_pmc.py PASS_DIR [PASS_DIR ...] --batch 4096 --blocks 2048 \
           --launch-blocks 512 --sr 48000 --chain 0 --lib tunebfree_amd/libtbf.so \
           --out profiles/kernel_pmc.json"""
import argparse
import csv
import hashlib
import json
import statistics
from collections import defaultdict
from pathlib import Path

FETCH_SCALE, WRITE_SCALE = 2.0, 1.0
# render stage -> kernel name prefix in the trace (stage 3 is the LDS network when it runs)
STAGES = (("k_tonegen", ("k_tonegen",)), ("k_mixpre", ("k_mixpre",)), ("k_rv_pre", ("k_rv_pre",)),
          ("k_rv_core", ("k_rv_core_lds", "k_rv_core")), ("k_rv_post", ("k_rv_post",)),
          ("k_whirl", ("k_whirl",)))


def stage_of(name):
    base = name.split("(")[0].replace("void ", "").split("<")[0].strip()
    for st, names in STAGES:
        if base in names:
            return st, base
    return None, base


def lib_hash(path):
    return hashlib.sha256(Path(path).read_bytes()).hexdigest()[:16]


def read_pass(d):
    """{(dispatch, stage, kernel, grid, ms): {counter: value}} of one pass directory"""
    f = Path(d) if Path(d).is_file() else next(Path(d).rglob("*counter_collection.csv"))
    out = defaultdict(lambda: defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(f)):
        st, kn = stage_of(r["Kernel_Name"])
        if st is None:
            continue
        k = int(r["Dispatch_Id"])
        out[k][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[k] = (st, kn, int(r["Grid_Size"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6,
                   int(r["VGPR_Count"]), int(r["Accum_VGPR_Count"]), int(r["LDS_Block_Size"]), int(r["Workgroup_Size"]))
    return out, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--blocks", type=int, default=2048)
    ap.add_argument("--launch-blocks", type=int, default=None, help="blocks per launch (default: --blocks)")
    ap.add_argument("--sr", type=float, default=48000.0)
    ap.add_argument("--chain", type=int, default=0)
    ap.add_argument("--lib", default="tunebfree_amd/libtbf.so")
    ap.add_argument("--out", default="profiles/kernel_pmc.json")
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(list))  # stage -> counter -> per-launch values (full launches)
    info, durs = {}, defaultdict(list)
    for d in a.dirs:
        vals, meta = read_pass(d)
        gmax = defaultdict(int)
        for st, kn, g, *_ in meta.values():
            gmax[st] = max(gmax[st], g)
        for k, cs in vals.items():
            st, kn, g, ms, vg, ag, lds, wg = meta[k]
            if g != gmax[st]:
                continue  # a smaller launch (parity-check engines, partial chunks)
            info[st] = {"kernel": kn, "grid": g, "workgroup": wg, "vgpr": vg, "agpr": ag, "lds_bytes": lds}
            durs[st].append(ms)
            for c, v in cs.items():
                per[st][c].append(v)
    lb = a.launch_blocks or a.blocks
    samples = a.batch * lb * 128
    res = {"build": lib_hash(a.lib), "lib": a.lib,
           "workload": {"batch": a.batch, "blocks": a.blocks, "sr": a.sr, "chain": a.chain},
           "launch_blocks": lb, "samples_per_launch": samples, "fetch_scale": FETCH_SCALE, "write_scale": WRITE_SCALE,
           "source": "rocprofv3 --pmc passes: " + ", ".join(a.dirs),
           "units": "per launch (median over full-size launches); FETCH/WRITE in bytes after the scale; "
                    "SQ_*_CYCLES and SQ_WAIT_*/SQ_ACTIVE_* in quad-cycles summed over waves; "
                    "GRBM_GUI_ACTIVE summed over the 8 XCDs",
           "kernels": {}}
    for st, _ in STAGES:
        if st not in per:
            continue
        c = {k: statistics.median(v) for k, v in per[st].items()}
        if "FETCH_SIZE" in c:
            c["FETCH_SIZE"] *= 1024.0 * FETCH_SCALE
        if "WRITE_SIZE" in c:
            c["WRITE_SIZE"] *= 1024.0 * WRITE_SCALE
        k = dict(info[st])
        k["launches"] = max(len(v) for v in per[st].values())
        k["pmc_ms"] = statistics.median(durs[st])
        k["counters"] = c
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            k["hbm_bytes"] = c["FETCH_SIZE"] + c["WRITE_SIZE"]
            k["hbm_bytes_per_stereo_sample"] = k["hbm_bytes"] / samples
        if "GRBM_GUI_ACTIVE" in c and k["pmc_ms"] > 0:
            k["clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / (k["pmc_ms"] * 1e-3) / 1e9
        res["kernels"][st] = k
        print(f"{st:10s} {k['kernel']:14s} n {k['launches']:2d} pmc {k['pmc_ms']:8.2f} ms  "
              + "  ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
