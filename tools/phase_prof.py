"""Per-segment wave-clock cycles per block of a kernel built by tools/phase_prof_patch.py
(segment k ends at the k-th sync of its device functions, in source order).
usage: TBF_LIB=<variant.so> python tools/phase_prof.py [--chain 0|1]"""
import argparse
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chain", type=int, default=0)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import tunebfree_amd as T
    wl = bench.Workload("cfg3", 48000.0)
    B, nb = 4096, int(os.environ.get("PROF_BLOCKS", "256"))
    eng = T.Engine(sample_rate=48000.0, device=0, chain=a.chain)
    bench.setup_instances(eng, wl, 0, B)
    outL = torch.empty((B, nb * 128), dtype=torch.float32, device="cuda")
    outR = torch.empty_like(outL)
    for _ in range(3):
        eng.render_device(nb, outL.data_ptr(), outR.data_ptr(), nb * 128, None)
        eng.synchronize()
    prof = outL[:8, :32].cpu().numpy().astype(np.float64) / nb
    tot = prof[:, 1:].sum(axis=1)
    for k in range(1, 32):
        if prof[:, k].max() > 0:
            print(f"segment {k:2d}  " + " ".join(f"{v:8.0f}" for v in prof[:, k]) + f"   ({np.mean(prof[:, k] / tot) * 100:4.1f} %)")
    print("total/block " + " ".join(f"{v:8.0f}" for v in tot))


if __name__ == "__main__":
    main()
