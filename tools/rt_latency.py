"""Real-time drop-in latency (§8(f) row 3): tbf_synth_sound for ONE instance, as an LV2
run() / CLAP process() callback would call it (b_synth/lv2.cpp:1056-1288,
src/clap.cpp:1128-1219), at 128- and 256-frame periods (48 kHz budgets 2.67 / 5.33 ms).

Each period: the events of that period (a chord change every 8 periods, a drawbar move
every 5), then tbf_synth_sound for the period's frames (the 128-sample FIFO renders a
block on the GPU when it runs dry: 5 stage kernels + copy-out + stream sync).  Wall
clock per call, p50 / p99 / max over the timed periods; a second pass retunes the
instance (tbf_instance_retune to a prebuilt 19-TET template) every 50 periods and
reports the retune periods apart.

    python tools/rt_latency.py [--periods N] [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pct(a, q):
    return float(np.percentile(np.asarray(a), q)) if len(a) else None


def run(frames, periods, warmup, retune_every, tunings):
    import tunebfree_amd as T
    import scenarios as S
    eng = T.Engine(sample_rate=48000.0, device=0)
    tid = eng.template(seed=7)
    tid19 = eng.template(mts128=np.asarray(tunings["19TET"], np.float64), seed=8)
    eng.add_instances([tid], [1000])
    for (k, a, v) in S.jazz1_params():
        eng.set_param(0, a, v)
    L = np.zeros(frames, np.float32)
    R = np.zeros(frames, np.float32)
    Lp, Rp = L.ctypes.data_as(T.engine._fp), R.ctypes.data_as(T.engine._fp)
    chords = [S.chord_for(i) for i in range(12)]
    held = []
    times, retune_times = [], []
    cur = tid
    for p in range(warmup + periods):
        t0 = time.perf_counter()
        if retune_every and p and p % retune_every == 0:
            cur = tid19 if cur == tid else tid
            eng.retune(0, cur)
            held = []  # the new tone generator starts with no keys down
        if p % 8 == 0:
            for k in held:
                eng.note(0, k, 0)
            held = chords[(p // 8) % 12]
            for k in held:
                eng.note(0, k, 1)
        if p % 5 == 0:
            eng.set_param(0, S.P_DRAWBAR + 3, (p // 5) % 9)
        rc = eng._lib.tbf_synth_sound(eng._h, frames, Lp, Rp, frames)
        assert rc == 0, rc
        dt = time.perf_counter() - t0
        if p >= warmup:
            (retune_times if retune_every and p % retune_every == 0 else times).append(dt * 1e3)
    eng.close()
    budget = frames / 48.0
    third = max(1, len(times) // 3)
    out = {"frames": frames, "budget_ms": budget, "periods": len(times), "p50_ms": pct(times, 50),
           "p99_ms": pct(times, 99), "max_ms": float(max(times)), "mean_ms": float(np.mean(times)),
           "over_budget": int(sum(t > budget for t in times)),
           # drift inside the run: the p50 of its first and last thirds (a clock ramp shows here)
           "p50_first_third_ms": pct(times[:third], 50), "p50_last_third_ms": pct(times[-third:], 50)}
    if retune_every:
        out.update({"retune_periods": len(retune_times), "retune_p50_ms": pct(retune_times, 50),
                    "retune_max_ms": float(max(retune_times)) if retune_times else None})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--periods", type=int, default=3000)
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--spin-ms", type=float, default=2000.0,
                    help="a full-size render loop before the rows, so the GPU and host clocks are up "
                         "(0: none -- the first row then pays the ramp)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")  # HIP runtime up before the engine (as bench.py)
    tunings = json.loads((ROOT / "tests" / "golden" / "tunings.json").read_text())
    import tunebfree_amd as T
    if a.spin_ms > 0:
        # the chip idles at a low clock: the first periods of a process ran at ~0.41 ms where
        # the same periods later take ~0.22 (round 4's rt_latency.json); spin it up first
        eng = T.Engine(sample_rate=48000.0, device=0)
        tid = eng.template(seed=7)
        eng.add_instances([tid] * 256, list(range(256)))
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < a.spin_ms:
            eng.render(64)
        eng.close()
    rows = []
    for frames in (128, 256):
        rows.append(run(frames, a.periods, a.warmup, 0, tunings))
        print(json.dumps(rows[-1]), flush=True)
        rows.append(dict(run(frames, a.periods, a.warmup, 50, tunings), mode="retune every 50 periods"))
        print(json.dumps(rows[-1]), flush=True)
    rows.append(dict(run(128, a.periods, a.warmup, 0, tunings), mode="128 frames again, last"))
    print(json.dumps(rows[-1]), flush=True)
    res = {"what": "tbf_synth_sound wall-clock per period, 1 instance, 48 kHz, full chain",
           "spin_ms": a.spin_ms, "warmup_periods": a.warmup,
           "host": os.uname().nodename, "gpu": torch.cuda.get_device_name(0), "rows": rows}
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
