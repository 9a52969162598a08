"""Steady render rate when the caller's stream is created before vs after the engine
(hardware-queue sharing: GPU_MAX_HW_QUEUES streams take the queues round-robin)."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def run(first):
    import torch
    import tunebfree_amd as T
    import scenarios as S
    B, nb = 4096, 64
    st = torch.cuda.Stream() if first else None
    eng = T.Engine(sample_rate=48000.0, device=0)
    if st is None:
        st = torch.cuda.Stream()
    tid = eng.template(seed=7)
    eng.add_instances([tid] * B, [1000 + i for i in range(B)])
    for i in range(B):
        for (_, kind, x, v) in S.bench_scenario(i):
            (eng.note if kind == "note" else eng.set_param)(i, x, v)
    L = torch.empty((B, nb * 128), dtype=torch.float32, device="cuda")
    R = torch.empty_like(L)
    for _ in range(3):
        eng.render_device(nb, L.data_ptr(), R.data_ptr(), nb * 128, st.cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        eng.render_device(nb, L.data_ptr(), R.data_ptr(), nb * 128, st.cuda_stream)
    st.synchronize()
    eng.synchronize()
    dt = (time.perf_counter() - t0) / 10
    print(f"caller stream created {'before' if first else 'after'} the engine: {dt * 1e3:.2f} ms per 64-block step", flush=True)
    eng.close()


if __name__ == "__main__":
    import torch
    torch.cuda.set_device(0)
    run(sys.argv[1] == "before")
