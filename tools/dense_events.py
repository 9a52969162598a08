"""Host control-plane cost under dense events (§8(f) rows 1-2): does the host's per-block
control stepping (message queue, active-oscillator list, routing, programme build:
src/tonegen.cpp:3257-3594 restated in tbf_init.cpp TgControl::step) show up in the step
time of the bench workload (configs[2]: 4096 instances, 64 blocks per step, Jazz-1 +
chord)?  One step = one tbf_render_events call of 64 blocks; modes:

  steady   no events inside the step (the bench's own line)
  every8   each instance changes its chord every 8 blocks (2 x 4 note events)
  dense    each instance releases one key and presses another on EVERY block
  params   each instance moves a drawbar on every block (no key change)
  sparseN  N instances (of the batch) change one note at the step's first block (2 N
           events: the size range of the device front end's event gate, TBF_FRONT_MIN)

For each: wall ms/step (HIP-synchronized), host control ms/step (tbf_debug_host_time),
time inside the tbf_render_events calls per step (host control + enqueueing + any wait),
events/step.  Writes JSON to --out.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def events_for(mode, B, blocks, step):
    import tunebfree_amd as T
    import scenarios as S
    ev = []
    if mode == "dense":
        out = np.zeros(blocks * B * 2, dtype=T.engine.EVENT_DTYPE)
        b = np.repeat(np.arange(blocks), B * 2)
        i = np.tile(np.repeat(np.arange(B), 2), blocks)
        on = np.tile([0.0, 1.0], blocks * B)
        t = step * blocks + b
        root = 48 + (i % 24)
        out["block"], out["inst"], out["kind"] = b, i, T.engine.EV_NOTE
        out["id"] = root + 14 + np.where(on > 0, t % 12, (t - 1) % 12)
        out["value"] = on
        return out
    elif mode == "every8":
        for b in range(0, blocks, 8):
            t = (step * blocks + b) // 8
            for i in range(B):
                for k in S.chord_for(i + t - 1):
                    ev.append((b, i, T.engine.EV_NOTE, k, 0.0))
                for k in S.chord_for(i + t):
                    ev.append((b, i, T.engine.EV_NOTE, k, 1.0))
    elif mode.startswith("sparse"):
        m = int(mode[6:])
        for i in range(m):
            j = (step * m + i) % B
            t = step
            ev.append((0, j, T.engine.EV_NOTE, 62 + (t - 1) % 12, 0.0))
            ev.append((0, j, T.engine.EV_NOTE, 62 + t % 12, 1.0))
        ev.sort(key=lambda r: r[0])
    elif mode == "params":
        for b in range(blocks):
            for i in range(B):
                ev.append((b, i, T.engine.EV_PARAM, S.P_DRAWBAR + 3, float((step * blocks + b + i) % 9)))
    return np.array(ev, dtype=T.engine.EVENT_DTYPE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--instances", type=int, default=4096)
    ap.add_argument("--blocks", type=int, default=64)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--modes", default="steady,every8,params,dense")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import tunebfree_amd as T
    import scenarios as S
    B, nb = a.instances, a.blocks
    rows = []
    for mode in a.modes.split(","):
        eng = T.Engine(sample_rate=48000.0, device=0)
        tid = eng.template(seed=7)
        eng.add_instances([tid] * B, [1000 + i for i in range(B)])
        for i in range(B):
            for (_, kind, x, v) in S.bench_scenario(i):
                (eng.note if kind == "note" else eng.set_param)(i, x, v)
        nsamp = nb * 128
        outL = torch.empty((B, nsamp), dtype=torch.float32, device="cuda")
        outR = torch.empty((B, nsamp), dtype=torch.float32, device="cuda")
        sptr = torch.cuda.current_stream().cuda_stream
        evs = [events_for(mode, B, nb, s) for s in range(a.warmup + a.steps)]
        for s in range(a.warmup):
            eng.render_events_device(nb, evs[s], outL.data_ptr(), outR.data_ptr(), nsamp, sptr)
        torch.cuda.synchronize()
        eng.synchronize()
        eng.host_time(reset=True)
        t0 = time.perf_counter()
        sub = 0.0
        for s in range(a.warmup, a.warmup + a.steps):
            ts = time.perf_counter()
            eng.render_events_device(nb, evs[s], outL.data_ptr(), outR.data_ptr(), nsamp, sptr)
            sub += time.perf_counter() - ts
        torch.cuda.synchronize()
        eng.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        hms, hblk = eng.host_time(reset=True)
        row = {"mode": mode, "instances": B, "blocks_per_step": nb, "events_per_step": int(len(evs[-1])),
               "ms_per_step": dt * 1e3, "host_control_ms_per_step": hms / a.steps,
               "call_ms_per_step": sub / a.steps * 1e3,
               "host_share": hms / a.steps / (dt * 1e3), "stereo_samples_per_s": B * nsamp / dt}
        rows.append(row)
        print(json.dumps(row), flush=True)
        eng.close()
        del outL, outR
    if a.out:
        Path(a.out).write_text(json.dumps({"what": "host control stepping under dense events", "rows": rows},
                                          indent=1) + "\n")


if __name__ == "__main__":
    main()
