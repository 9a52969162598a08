#!/usr/bin/env python3
"""Measure the VALU issue cost bench.py's roofline assumes.

tbf_debug_calibrate ops 5..12 (csrc/tbf_calib.hip) run 2048 workgroups of 4 waves (8 waves
per SIMD on 256 CUs), each wave 32 x iters instructions of one kind in 8 independent chains
(inline asm), so every SIMD is issue-bound.  The launch is timed with HIP events on its
stream, the shader clock comes from the kernel itself (s_memtime cycles over s_memrealtime
ticks at 100 MHz), and

    cycles per wave64 instruction per SIMD = time x clock / (8 waves x 32 iters)

Writes a JSON (default profiles/valu_calib.json) that bench.py reads for VALU_CYC.
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

OPS = [("v_add_f32", "base"), ("v_fma_f32", "fma32"), ("v_add_f64", "f64"), ("v_mul_f64", "mul64"),
       ("v_fma_f64", "fma64"), ("v_sin_f32", "trans32"), ("v_rcp_f64", "trans64"), ("v_add_u32", "int")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=4000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=str(ROOT / "profiles" / "valu_calib.json"))
    a = ap.parse_args()
    import ctypes as C
    import torch
    import tunebfree_amd as T
    lib = T.load_library()
    fn = lib.tbf_debug_calibrate
    fn.restype, fn.argtypes = C.c_int, [C.c_int32, C.c_void_p, C.c_uint64, C.c_void_p]
    torch.cuda.set_device(0)
    buf = torch.zeros(2 + 4096, dtype=torch.float64, device="cuda")
    st = torch.cuda.Stream()
    waves_per_simd, per_trip = 8, 32
    rows = {}
    for k, (ins, key) in enumerate(OPS):
        op = 5 + k
        with torch.cuda.stream(st):
            assert fn(op, buf.data_ptr(), a.iters, st.cuda_stream) == 0  # warm-up (clock ramp, code load)
            st.synchronize()
            best = None
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                assert fn(op, buf.data_ptr(), a.iters, st.cuda_stream) == 0
                e1.record(st)
                st.synchronize()
                ms = e0.elapsed_time(e1)
                cyc, ticks = float(buf[0].item()), float(buf[1].item())
                ghz = cyc / (ticks / 100e6) / 1e9 if ticks else float("nan")
                cpi = ms * 1e-3 * ghz * 1e9 / (waves_per_simd * per_trip * a.iters)
                r = {"ms": ms, "clock_ghz": ghz, "cycles_per_wave64_inst": cpi}
                if best is None or ms < best["ms"]:
                    best = r
        rows[key] = dict(best, instruction=ins)
        print(f"{ins:10s} {best['ms']:8.3f} ms  clock {best['clock_ghz']:.3f} GHz  "
              f"{best['cycles_per_wave64_inst']:.2f} cycles / wave64 instruction / SIMD", flush=True)
    res = {"source": "tools/valu_calib.py (tbf_debug_calibrate ops 5..12)", "iters": a.iters,
           "waves_per_simd": waves_per_simd, "device": torch.cuda.get_device_name(0),
           "date": time.strftime("%Y-%m-%d %H:%M"), "ops": rows,
           "valu_cyc": {"base": rows["base"]["cycles_per_wave64_inst"],
                        "f64": max(rows["f64"]["cycles_per_wave64_inst"], rows["mul64"]["cycles_per_wave64_inst"],
                                   rows["fma64"]["cycles_per_wave64_inst"]),
                        "trans32": rows["trans32"]["cycles_per_wave64_inst"],
                        "trans64": rows["trans64"]["cycles_per_wave64_inst"]}}
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))
    print(json.dumps(res["valu_cyc"]))


if __name__ == "__main__":
    main()
