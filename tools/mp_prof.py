"""k_mixpre role / section clocks (profiling variant MP_PROF=1, never the product): the
bench's batch and registration in the preamp-tap chain mode, one 512-block launch after a
warm-up launch; workgroup 0's serial, dither and first helper waves write their s_memtime
sums (k cycles) over instance 0's first output samples.

    TBF_LIB=tunebfree_amd/_variants/libtbf_mpprof.so python tools/mp_prof.py"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    import torch
    import tunebfree_amd as T
    import scenarios as S
    B, nb = 4096, 512  # one steady-chunk launch
    eng = T.Engine(sample_rate=48000.0, device=0, chain=2)
    tid = eng.template(seed=7)
    eng.add_instances([tid] * B, [1000 + i for i in range(B)])
    for i in range(B):
        for (_, kind, a, v) in S.bench_scenario(i):
            (eng.note if kind == "note" else eng.set_param)(i, a, v)
    L = torch.empty((B, nb * 128), dtype=torch.float32, device="cuda")
    R = torch.empty_like(L)
    for _ in range(2):
        eng.render_device(nb, L.data_ptr(), R.data_ptr(), nb * 128)
        eng.synchronize()
    v = L[0, :64].cpu().numpy()
    it = nb * 2 + 3  # 64-sample tiles (MP_WIDE), two per block
    print(f"per iteration (cycles), {it} iterations:")
    print(f"  helper 0: waveshaper {v[0] * 1e3 / it:8.0f}  products+loads {v[1] * 1e3 / it:8.0f}  barrier {v[2] * 1e3 / it:8.0f}")
    print(f"  serial  : work       {v[8] * 1e3 / it:8.0f}  barrier        {v[9] * 1e3 / it:8.0f}")
    print(f"  dither  : work       {v[16] * 1e3 / it:8.0f}  barrier        {v[17] * 1e3 / it:8.0f}")
    print(f"  (serial on SIMD {v[10]:.0f}, dither on SIMD {v[18]:.0f})")
    for h in range(8):
        b = 32 + 4 * h
        print(f"  helper {h} (SIMD {v[b + 3]:.0f}): waveshaper {v[b] * 1e3 / it:8.0f}  products+loads {v[b + 1] * 1e3 / it:8.0f}"
              f"  barrier {v[b + 2] * 1e3 / it:8.0f}")


if __name__ == "__main__":
    main()
