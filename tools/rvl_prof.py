"""Per-segment wave-clock cycles of k_rv_core_lds from a build made by
tools/rvl_prof_patch.py: the bench workload (4096 instances, 64 blocks per step) rendered
with pipelining off (each kernel alone), cycles per (instance, channel) pair and per group.
usage: TBF_LIB=<variant.so> python tools/rvl_prof.py"""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

SEGS = ["pair start/ring load", "pre-loop barrier", "read phase", "barrier 1", "write phase", "barrier 2",
        "ring store", "groups"]


def main():
    import numpy as np
    import torch
    import bench
    import tunebfree_amd as T
    wl = bench.Workload("cfg3", 48000.0)
    B, nb, steps = 4096, int(os.environ.get("PROF_BLOCKS", "256")), 3
    eng = T.Engine(sample_rate=48000.0, device=0)
    bench.setup_instances(eng, wl, 0, B)
    lib = T.load_library()
    fn = lib.tbf_debug_rvl_prof
    fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_int]
    outL = torch.empty((B, nb * 128), dtype=torch.float32, device="cuda")
    outR = torch.empty_like(outL)
    buf = np.zeros((16, 8), np.uint64)
    eng.kernel_times("serial")
    for _ in range(2):
        eng.render_device(nb, outL.data_ptr(), outR.data_ptr(), nb * 128, None)
    eng.synchronize()
    assert fn(buf.ctypes.data, 1) == 0
    for _ in range(steps):
        eng.render_device(nb, outL.data_ptr(), outR.data_ptr(), nb * 128, None)
    eng.synchronize()
    kt = eng.kernel_times()
    assert fn(buf.ctypes.data, 0) == 0
    pairs = 2 * B * steps
    print("k_rv_core ms alone:", {k: round(v[0] / v[1], 3) for k, v in kt.items() if v[1]})
    print("cycles per pair (rows: wave 0..11, 11 = planner); groups per pair", buf[0, 7] / pairs)
    print("wave " + "".join(f"{s[:14]:>16s}" for s in SEGS[:7]) + "           total")
    for w in range(12):
        r = buf[w, :7].astype(np.float64) / pairs
        print(f"{w:4d} " + "".join(f"{v:16.0f}" for v in r) + f"{r.sum():16.0f}")
    g = buf[0, 7] / pairs
    print("per group (wave 0): " + ", ".join(f"{SEGS[k]} {buf[0, k] / pairs / g:.0f}" for k in (2, 3, 4, 5)))
    print("per group (planner): " + ", ".join(f"{SEGS[k]} {buf[11, k] / pairs / g:.0f}" for k in (2, 3, 4, 5)))


if __name__ == "__main__":
    main()
