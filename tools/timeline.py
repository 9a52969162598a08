"""Concurrency profile of the rendered chain from a rocprofv3 --kernel-trace CSV: over the
window of full-size launches after the warmup, the wall time by the SET of stage kernels
running at each instant (which kernels overlap, and for how long each runs alone), plus
each kernel's mean duration as rendered.  Tells which stream is the critical path and how
much of a kernel's time other stages fill.

usage: python tools/timeline.py KERNEL_TRACE_CSV [--skip-ms MS] [--out JSON]"""
import argparse
import csv
import json
from collections import defaultdict

SHORT = {"k_tonegen": "tg", "k_mixpre": "mp", "k_rv_pre": "pre", "k_rv_core_lds": "core", "k_rv_core": "core",
         "k_rv_post": "post", "k_whirl": "wh", "k_tgctl": "ctl", "k_front": "front"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip-ms", type=float, default=None, help="ignore launches starting before this (default: first 30 %%)")
    ap.add_argument("--out")
    a = ap.parse_args()
    ev = []
    gmax = defaultdict(int)
    for r in csv.DictReader(open(a.trace)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
        if name not in SHORT:
            continue
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, grid))
        gmax[name] = max(gmax[name], grid)
    ev = [e for e in ev if e[3] == gmax[e[2]]]  # full-size launches only
    ev.sort()
    t0 = ev[0][0]
    tend = max(e[1] for e in ev)
    skip = a.skip_ms * 1e6 if a.skip_ms is not None else 0.3 * (tend - t0)
    ev = [e for e in ev if e[0] - t0 >= skip]
    w0, w1 = ev[0][0], max(e[1] for e in ev)
    pts = sorted([(s, 1, n) for s, _, n, _ in ev] + [(e, -1, n) for _, e, n, _ in ev])
    active = defaultdict(int)
    by_set = defaultdict(float)
    alone = defaultdict(float)
    last = w0
    for t, d, n in pts:
        if t > last:
            key = "+".join(sorted(SHORT[k] for k, c in active.items() if c > 0)) or "idle"
            by_set[key] += (t - last) * 1e-6
            run = [k for k, c in active.items() if c > 0]
            if len(run) == 1:
                alone[run[0]] += (t - last) * 1e-6
            last = t
        active[n] += d
    total = (w1 - w0) * 1e-6
    dur = defaultdict(list)
    for s, e, n, _ in ev:
        dur[n].append((e - s) * 1e-6)
    print(f"window {total:.1f} ms, {len(ev)} launches")
    for k, v in sorted(by_set.items(), key=lambda x: -x[1])[:20]:
        print(f"  {k:28s} {v:9.2f} ms  {100 * v / total:5.1f} %")
    print("per kernel: mean as rendered, launches, ms running alone")
    out = {"window_ms": total, "by_set_ms": by_set, "kernels": {}}
    for n, v in sorted(dur.items()):
        m = sum(v) / len(v)
        print(f"  {n:16s} {m:8.3f} ms  x{len(v):3d}  alone {alone[n]:8.2f} ms")
        out["kernels"][n] = {"mean_ms": m, "launches": len(v), "alone_ms": alone[n]}
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
