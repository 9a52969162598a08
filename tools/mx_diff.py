"""tools/mx_diff.py -- the first keys whose play-matrix lists differ between the device
builder (tbf_templates_create) and the host one (tbf_template_create), for one tuning."""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import tunebfree_amd as T  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "19TET"
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 301
tun = json.loads((ROOT / "tests" / "golden" / "tunings.json").read_text())
m = None if tun[name] is None else np.asarray(tun[name], np.float64)
lib = T.load_library()
lib.tbf_debug_contrib.restype = C.c_int
lib.tbf_debug_contrib.argtypes = [C.c_void_p, C.c_uint32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]
eng = T.Engine(sample_rate=48000.0, device=0)
d = eng.templates([seed], mts128=None if m is None else m[None])[0]
h = eng.template(mts128=m, seed=seed)


def lst(t, k):
    w, b, lv = np.zeros(4096, np.int16), np.zeros(4096, np.int16), np.zeros(4096, np.float32)
    c = lib.tbf_debug_contrib(eng._h, t, k, w.ctypes.data, b.ctypes.data, lv.ctypes.data, 4096)
    return [(int(w[i]), int(b[i]), float(lv[i])) for i in range(c)]


bad = 0
for k in range(384):
    a, b = lst(d, k), lst(h, k)
    if a != b:
        bad += 1
        if bad <= 4:
            print(f"key {k}: device {len(a)} host {len(b)}")
            sa, sb = set(a), set(b)
            print("  device only:", sorted(sa - sb)[:12])
            print("  host only:  ", sorted(sb - sa)[:12])
            if sa == sb:
                print("  order differs:", a[:8], b[:8])
print(f"{bad} of 384 keys differ")
eng.close()
