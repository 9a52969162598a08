"""Summarize a bench.py JSON line (optionally with --isolated): step, parity, per-kernel times.
usage: python tools/isosum.py LOG [LOG ...]"""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        r = d.get("roofline") or {}
        print(f"{f}: {d['value']:.4g} stereo samples/s, {d['ms_per_step']:.3f} ms/step, "
              f"max_err {d.get('max_err')}, exact {d.get('bit_exact_frac')}")
        for key in ("kernels_ms_per_launch", "kernels_ms_isolated"):
            if r.get(key):
                print(f"  {key[8:]:>16}: " + "  ".join(f"{k} {v:.3f}" for k, v in r[key].items()))
