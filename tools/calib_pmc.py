"""Known-byte streams for FETCH_SIZE / WRITE_SIZE calibration (run under rocprofv3 --pmc).
Streams N doubles (default 2 GiB, far beyond the 256 MiB MALL) with the render kernel's
8-B/lane pattern: 3 read launches then 3 write launches.
usage: rocprofv3 --pmc FETCH_SIZE -- python3 tools/calib_pmc.py [GiB] [ops, e.g. 0,2,1,3: 2/3 = misaligned by 64 B]"""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
    import torch
    import tunebfree_amd as T
    lib = T.load_library()
    lib.tbf_debug_calibrate.restype = C.c_int
    lib.tbf_debug_calibrate.argtypes = [C.c_int32, C.c_void_p, C.c_uint64, C.c_void_p]
    n = int(gib * (1 << 30)) // 8
    buf = torch.zeros(n, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    ops = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 0, 0, 1, 1, 1]
    for op in ops:
        assert lib.tbf_debug_calibrate(op, C.c_void_p(buf.data_ptr()), n, None) == 0
    torch.cuda.synchronize()
    print(f"calibration: {n} doubles = {n * 8} bytes per launch")


if __name__ == "__main__":
    main()
