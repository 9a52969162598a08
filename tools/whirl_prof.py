"""Per-phase wave-clock cycles of k_whirl (profiling variant from tools/whirl_prof_patch.py):
renders the bench workload with TBF_LIB pointing at the variant and prints each phase's
cycles per block for instances 0..7.  usage: TBF_LIB=... python tools/whirl_prof.py"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

NAMES = {10: "block start", 9: "speed (lane 0)", 1: "ring read + staging", 3: "serial filters", 4: "filter outputs + angles",
         5: "FILTER_C", 6: "motions (tables)", 7: "ring adds", 8: "outputs + carry"}


def main():
    import numpy as np
    import torch
    import bench
    import tunebfree_amd as T
    wl = bench.Workload("cfg3", 48000.0)
    B, nb = 4096, int(os.environ.get("PROF_BLOCKS", "256"))
    eng = T.Engine(sample_rate=48000.0, device=0)
    bench.setup_instances(eng, wl, 0, B)
    outL = torch.empty((B, nb * 128), dtype=torch.float32, device="cuda")
    outR = torch.empty_like(outL)
    for _ in range(3):
        eng.render_device(nb, outL.data_ptr(), outR.data_ptr(), nb * 128, None)
        eng.synchronize()
    prof = outL[:8, :16].cpu().numpy()
    tot = prof[:, [k for k in NAMES]].sum(axis=1)
    for k, nm in NAMES.items():
        print(f"{nm:26s} " + " ".join(f"{v / nb:8.0f}" for v in prof[:, k]) + f"   ({np.mean(prof[:, k] / tot) * 100:4.1f} %)")
    print(f"{'total per block':26s} " + " ".join(f"{v / nb:8.0f}" for v in tot))


if __name__ == "__main__":
    main()
