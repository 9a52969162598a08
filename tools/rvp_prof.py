"""k_rv_post role clocks (profiling variant RVP_PROF=1, never the product): the bench's batch
and registration in the reverb-tap chain mode, one 512-block launch after warm-up launches;
workgroup 0's serial, dither and first helper waves write their s_memtime sums (k cycles) of
work and barrier wait over instance 0's first output samples.

    TBF_LIB=tunebfree_amd/_variants/libtbf_rvpprof.so python tools/rvp_prof.py"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    import torch
    import tunebfree_amd as T
    import scenarios as S
    B, nb = 4096, 512
    eng = T.Engine(sample_rate=48000.0, device=0, chain=3)
    tid = eng.template(seed=7)
    eng.add_instances([tid] * B, [1000 + i for i in range(B)])
    for i in range(B):
        for (_, kind, a, v) in S.bench_scenario(i):
            (eng.note if kind == "note" else eng.set_param)(i, a, v)
    L = torch.empty((B, nb * 128), dtype=torch.float32, device="cuda")
    R = torch.empty_like(L)
    for _ in range(3):
        eng.render_device(nb, L.data_ptr(), R.data_ptr(), nb * 128)
        eng.synchronize()
    v = L[0, :64].cpu().numpy()
    it = nb * 4 + 4
    print(f"k_rv_post per iteration (cycles), {it} iterations:")
    for name, o in (("serial", 0), ("dither", 4), ("helper0", 8)):
        print(f"  {name:8s} work {v[o] * 1e3 / it:8.0f}  barrier {v[o + 1] * 1e3 / it:8.0f}")
    print("every wave of workgroup 0 (wave: work / barrier cycles per iteration, SIMD):")
    for w in range(11):
        b = 16 + 3 * w
        print(f"  wave {w:2d}: {v[b] * 1e3 / it:8.0f} / {v[b + 1] * 1e3 / it:8.0f}  SIMD {v[b + 2]:.0f}")


if __name__ == "__main__":
    main()
