"""Per-stage wave-clock breakdown of the render kernel (tbf_debug_profile marks).
usage: python tools/prof_stages.py [--batch 4096] [--blocks 32]
The marks are compiled only into a profiling build (the product kernels keep that LDS free):
  make -C tunebfree_amd variant NAME=prof VFLAGS=-DTBF_STAGE_PROF=1
  TBF_LIB=tunebfree_amd/_variants/libtbf_prof.so python tools/prof_stages.py
Marks add a workgroup barrier each, so totals run ~10% above the unprofiled kernel."""
import argparse
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

NAMES = {0: "tg state load + interpreter", 1: "tg vibrato", 2: "tg mixdown", 3: "od dither + HPF chain",
         4: "od waveshaper", 18: "tg state store",
         5: "rv_in dither", 6: "rv_in predelay + biquadA chain", 7: "rv_in sin(x*wet)",
         8: "rv_core channel L", 9: "rv_core channel R + counts",
         10: "rv_out load", 11: "rv_out B(b) + C(b-1) chains", 12: "rv_out dither + dry + store",
         13: "rv_out asin",
         14: "rv_lds ring load", 15: "rv_lds plan", 16: "rv_lds read phase", 17: "rv_lds write phase",
         19: "rv_lds ring store",
         26: "wh state + ring load", 20: "wh speed", 21: "wh ring rd + serial filt+angles", 22: "wh FILTER_C",
         23: "wh motions", 24: "wh accumulate", 25: "wh out + carry", 27: "wh state + ring store"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--blocks", type=int, default=32)
    a = ap.parse_args()
    import torch
    import tunebfree_amd as T
    import scenarios as S
    eng = T.Engine(sample_rate=48000.0, device=0)
    tid = eng.template(seed=7)
    B = a.batch
    eng.add_instances([tid] * B, [1000 + i for i in range(B)])
    for i in range(B):
        for (_, kind, x, v) in S.bench_scenario(i):
            (eng.note if kind == "note" else eng.set_param)(i, x, v)
    n = a.blocks * 128
    oL = torch.empty((B, n), dtype=torch.float32, device="cuda")
    oR = torch.empty((B, n), dtype=torch.float32, device="cuda")
    eng.render_device(a.blocks, oL.data_ptr(), oR.data_ptr(), n)
    eng.synchronize()
    lib = T.load_library()
    lib.tbf_debug_profile.restype = C.c_int
    lib.tbf_debug_profile.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_uint32]
    assert lib.tbf_debug_profile(eng._h, 1, None, 0) == 0
    eng.render_device(a.blocks, oL.data_ptr(), oR.data_ptr(), n)
    eng.synchronize()
    buf = np.zeros(B * 32, np.uint64)
    assert lib.tbf_debug_profile(eng._h, 0, buf.ctypes.data, buf.size) >= 0
    lib.tbf_debug_profile(eng._h, -1, None, 0)
    per = buf.reshape(B, 32).astype(np.float64).mean(axis=0) / a.blocks
    tot = per.sum()
    print(f"wave-clock cycles per 128-sample block (mean over {B} instances), total {tot:.0f}")
    for k in range(32):
        if per[k] > 0:
            print(f"  {k:2d} {NAMES.get(k, '?'):28s} {per[k]:10.0f}  {100 * per[k] / tot:5.1f}%")


if __name__ == "__main__":
    main()
