#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: stereo samples/sec whole-node, full chain
(tonegen -> vibrato -> overdrive -> reverb -> whirl) at 48 kHz, 4096 organ instances
per GPU (configs[2] at N=1; configs[3] = 8 x 4096 at N=8, weak scaling), with
max|err| vs the CPU chain.

A "step" is one kernel pass over the batch: every instance renders `--blocks`
128-sample blocks (default 64 = 8192 stereo samples per instance).  Inputs are
synthetic: instance i plays the "Jazz 1 all" registration (pgm/default.pgm:27-36)
with overdrive character 0.5, reverb 0.1, rotary chorale, chord root 48+(i mod 24)
+ {0,4,7,12}; note-on lands at block 0 of the first warmup step.

Launch: python bench.py --gpus N --steps K --warmup W   (N>1 under torch.distributed.run,
one rank per GPU; instances shard across ranks, no data-path collective).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

# algorithmic HBM bytes per stereo sample, per kernel:
#   k_rv_core = 12 lines x 2 ch x (8 B write + 8 B read) ring streaming + 16 B in + 16 B out
#   k_rv_in   = predelay ring 2 ch x 16 B + 4 B in + 16 B out
#   k_rv_out  = 16 B tap mix + 4 B dry in + 4 B out
#   k_tonegen = 4 B stage output (wave bank L2/MALL-resident)
#   k_whirl   = 4 B in + 8 B L/R out
ALGO_BYTES = {"k_tonegen": 4, "k_rv_in": 52, "k_rv_core": 416, "k_rv_out": 24, "k_whirl": 12}
DOMINANT = "k_rv_core"  # the HBM-streaming kernel the roofline is quoted for
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
TRAFFIC_JSON = ROOT / "profiles" / "traffic.json"  # written by tools/traffic_from_pmc.py


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096, help="instances per GPU")
    ap.add_argument("--blocks", type=int, default=64, help="128-sample blocks per step")
    ap.add_argument("--sr", type=float, default=None, help="sample rate (default 48000; 96000 for cfg5)")
    ap.add_argument("--workload", choices=("cfg3", "cfg2", "cfg5"), default="cfg3",
                    help="cfg3: BASELINE configs[2]/[3] (the metric's workload); cfg2: configs[1] (tonegen only, "
                         "use with --batch 256); cfg5: configs[4] per-GPU sub-batch (96 kHz, 7 tunings, random "
                         "drawbars) -- secondary lines, not the headline")
    ap.add_argument("--check", type=int, default=4, help="instances checked against the CPU oracle")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-instances", type=int, default=128)
    ap.add_argument("--cpu-blocks", type=int, default=12000)
    ap.add_argument("--chain", type=int, default=0, help="0 full chain; 1/2/3 stage taps (profiling only)")
    ap.add_argument("--isolated", type=int, default=0,
                    help="also time each kernel alone (pipelining off); adds launches to a profiled run")
    ap.add_argument("--traffic", default=str(TRAFFIC_JSON), help="PMC traffic JSON (tools/traffic_from_pmc.py)")
    ap.add_argument("--kernel-steps", type=int, default=None,
                    help="extra steps timed per kernel with HIP events for the roofline (default = --steps)")
    return ap.parse_args()


class Workload:
    """Per-instance template, seed and event script of a BASELINE config.
    cfg3: configs[2]/[3] (one 48 kHz template, seed 7; Jazz-1 + chord per instance).
    cfg2: configs[1] (tonegen only: chain mode 1, L = R = oscGenerateFragment; drawbars
    888000000 + vibrato, the same chords).
    cfg5: configs[4] (one shared template per tuning of tests/golden/tunings.json,
    instance g on tuning (5 g) mod 7, randomizeDrawbars-style upper drawbars)."""

    def __init__(self, kind, sr):
        import scenarios as S
        self.kind, self.sr, self.S = kind, sr, S
        self.names = [None]
        self.mts = {None: None}
        if kind == "cfg5":
            import numpy as np
            tun = json.loads((ROOT / "tests" / "golden" / "tunings.json").read_text())
            self.names = sorted(tun, key=lambda k: (tun[k] is not None, k))
            self.mts = {nm: (None if tun[nm] is None else np.array(tun[nm], np.float64)) for nm in self.names}

    def tpl_seed(self, j):
        return 100 + j if self.kind == "cfg5" else 7

    def tuning_of(self, g):
        return (5 * g) % len(self.names) if self.kind == "cfg5" else 0

    def seed_of(self, g):
        return 1000 + g

    def scenario(self, g):
        if self.kind == "cfg5":
            return self.S.random_drawbar_scenario(g)
        return self.S.bench_scenario(g, full=self.kind == "cfg3")

    def describe(self, B, world, blocks):
        if self.kind == "cfg2":
            return (f"configs[1]: tonegen only (oscGenerateFragment + vibrato, L = R), {B} instances/GPU x "
                    f"{world} GPU(s), {self.sr:.0f} Hz, {blocks} blocks/step, drawbars 888000000 + 4-note chords")
        if self.kind == "cfg3":
            return (f"configs[{2 if world == 1 else 3}]: full chain tonegen->vibrato->overdrive->reverb->whirl, "
                    f"{B} instances/GPU x {world} GPU(s), {self.sr:.0f} Hz, {blocks} blocks/step, "
                    f"Jazz-1 registration + 4-note chords")
        return (f"configs[4] per-GPU sub-batch: full chain, {B} instances/GPU x {world} GPU(s), {self.sr:.0f} Hz, "
                f"{len(self.names)} tunings (one shared bank each), random upper drawbars, {blocks} blocks/step")


def setup_instances(eng, wl, first_global, n):
    tids = [eng.template(mts128=wl.mts[nm], seed=wl.tpl_seed(j)) for j, nm in enumerate(wl.names)]
    eng.add_instances([tids[wl.tuning_of(first_global + i)] for i in range(n)],
                      [wl.seed_of(first_global + i) for i in range(n)])
    for i in range(n):
        for (_, kind, a, v) in wl.scenario(first_global + i):
            if kind == "note":
                eng.note(i, a, v)
            else:
                eng.set_param(i, a, v)


def _cpu_worker(args):
    """CPU render of a slice of instances; returns samples and seconds.  kind "reference":
    the reference's own tonegen/vibrato/overdrive/reverb/whirl translation units compiled
    by oracle/Makefile (oracle/_ref/libtbfref.so), driven like synthSound; kind "port":
    the oracle's C restatement."""
    idx, blocks, sr, kind = args
    import scenarios as S
    from orc_bind import Chain, Template, load_oracle, load_ref
    lib = load_oracle()
    ref = load_ref() if kind == "reference" else None
    tpl = Template(lib, sr=sr, seed=7)
    chains = []
    for i in idx:
        ch = Chain(ref, tpl, 1000 + i, ref=True) if ref is not None else Chain(lib, tpl, 1000 + i)
        for (_, kind, a, v) in S.bench_scenario(i):
            (ch.note if kind == "note" else ch.param)(a, v)
        chains.append(ch)
    t0 = time.perf_counter()
    for ch in chains:
        ch.render(blocks)
    return len(idx) * blocks * 128, time.perf_counter() - t0


def cpu_baseline(n_inst, blocks, sr):
    import multiprocessing as mp
    kind = "reference" if (ROOT / "oracle" / "_ref" / "libtbfref.so").exists() else "port"
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16, n_inst))
    parts = [list(range(k, n_inst, cores)) for k in range(cores)]
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(cores) as pool:
        res = pool.map(_cpu_worker, [(p, blocks, sr, kind) for p in parts])
    wall = time.perf_counter() - t0
    samples = sum(r[0] for r in res)
    busy = max(r[1] for r in res)  # render time of the slowest worker (construction excluded)
    what = ("the reference's src/tonegen.cpp, vibrato.cpp, overdrive.cpp, reverb.cpp, whirl.cpp "
            "compiled by oracle/Makefile (gcc -O2)" if kind == "reference" else "oracle/ C restatement")
    return {"value": samples / busy, "unit": "stereo samples/s", "cores": cores, "kind": kind,
            "sample": f"{n_inst} instances x {blocks} blocks ({blocks * 128 / sr:.2f} s audio each), "
                      f"{what}, {cores} processes, construction excluded (wall {wall:.1f}s)"}


def oracle_check(wl, rank_first, n_check, total_blocks, last_blocks, gpu_L, gpu_R):
    """max|err| of the last step's outputs vs the CPU oracle for the first instances."""
    import numpy as np
    from orc_bind import Chain, Template, load_oracle
    lib = load_oracle()
    tpls = {}
    err, exact, tot = 0.0, 0, 0
    for i in range(n_check):
        g = rank_first + i
        j = wl.tuning_of(g)
        if j not in tpls:
            tpls[j] = Template(lib, sr=wl.sr, mts128=wl.mts[wl.names[j]], seed=wl.tpl_seed(j))
        ch = Chain(lib, tpls[j], wl.seed_of(g))
        if wl.kind == "cfg2":
            ch.chain(1)
        for (_, kind, a, v) in wl.scenario(g):
            (ch.note if kind == "note" else ch.param)(a, v)
        ch.render(total_blocks - last_blocks)
        L, R = ch.render(last_blocks)
        for x, y in ((gpu_L[i], L), (gpu_R[i], R)):
            d = np.abs(x.astype(np.float64) - y.astype(np.float64))
            err = max(err, float(d.max()))
            exact += int(np.sum(x.view(np.uint32) == y.view(np.uint32)))
            tot += x.size
    return err, exact / max(tot, 1)


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    else:
        torch.cuda.set_device(0)
    import tunebfree_amd as T

    B = a.batch
    first_global = rank * B
    if a.sr is None:
        a.sr = 96000.0 if a.workload == "cfg5" else 48000.0
    wl = Workload(a.workload, a.sr)
    if a.workload == "cfg2":
        a.chain = 1  # TBF_CHAIN_TONEGEN
    eng = T.Engine(sample_rate=a.sr, device=torch.cuda.current_device(), chain=a.chain)
    setup_instances(eng, wl, first_global, B)
    nsamp = a.blocks * 128
    outL = torch.empty((B, nsamp), dtype=torch.float32, device="cuda")
    outR = torch.empty((B, nsamp), dtype=torch.float32, device="cuda")
    stream = torch.cuda.Stream()  # a real stream: the kernel and the timing events share it
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream

    def step():
        eng.render_device(a.blocks, outL.data_ptr(), outR.data_ptr(), nsamp, sptr)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    t0 = time.perf_counter()
    for k in range(a.steps):
        ev[k][0].record(stream)
        step()
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    total_samples = world * B * nsamp * a.steps
    value = total_samples / elapsed

    # per-kernel launch durations (HIP events on each launch's stream, inside the
    # engine), rendered exactly like the timed region (cross-chunk pipelining on, so a
    # duration includes the overlap with the neighbouring chunk's kernels); a separate
    # pass so the events do not perturb the timed region above
    ksteps = a.steps if a.kernel_steps is None else a.kernel_steps
    eng.kernel_times(True)
    for _ in range(ksteps):
        step()
    torch.cuda.synchronize()
    kt = eng.kernel_times()
    eng.kernel_times(False)
    kern = {k: v[0] / v[1] for k, v in kt.items() if v[1]}
    kern_iso = None
    if a.isolated:  # each kernel alone on the GPU (pipelining off): per-kernel tuning
        eng.kernel_times("serial")
        for _ in range(ksteps):
            step()
        torch.cuda.synchronize()
        kt = eng.kernel_times()
        eng.kernel_times(False)
        kern_iso = {k: v[0] / v[1] for k, v in kt.items() if v[1]}

    # parity on the last step (first --check instances of this rank)
    gL = outL[: a.check].cpu().numpy()
    gR = outR[: a.check].cpu().numpy()
    total_blocks = (a.warmup + a.steps + ksteps * (2 if a.isolated else 1)) * a.blocks
    max_err, exact = oracle_check(wl, first_global, a.check, total_blocks, a.blocks, gL, gR) if a.check else (None, None)
    if dist:
        e = torch.tensor([max_err or 0.0], dtype=torch.float64, device="cuda")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        max_err = float(e.item())

    if rank == 0:
        samples_launch = B * nsamp
        if a.chain == 1:  # tonegen only: k_tonegen writes L and R (8 B); bank reads are L2-resident
            ALGO_BYTES["k_tonegen"] = 8
        dom = DOMINANT if DOMINANT in kern else max(kern, key=kern.get)
        achieved = samples_launch * ALGO_BYTES[dom] / (kern[dom] * 1e-3) / 1e9
        traffic, traffic_src = None, None
        if Path(a.traffic).exists():
            tj = json.loads(Path(a.traffic).read_text())
            if tj.get("workload") == {"batch": B, "blocks": a.blocks, "sr": a.sr, "chain": a.chain} \
                    and dom in tj.get("kernels", {}):
                traffic = tj["kernels"][dom]["bytes_per_launch"]
                traffic_src = tj.get("source")
        cpu = cpu_baseline(a.cpu_instances, a.cpu_blocks, a.sr) if (a.cpu_baseline and world == 1 and a.workload == "cfg3") else None
        line = {
            "metric": "stereo samples/sec whole-node, batch=4096 full chain @48kHz; max|err| vs CPU",
            "value": value, "unit": "stereo samples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32 (f64 reverb/overdrive)", "data": "synthetic",
            "config": {"workload": wl.describe(B, world, a.blocks),
                       "batch_per_gpu": B, "blocks_per_step": a.blocks, "sample_rate": a.sr,
                       "parallelism": f"instance-sharded x{world} (no collective)"},
            "max_err": max_err, "bit_exact_frac": exact, "checked_instances": a.check,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": dom, "kernel_ms_per_launch": kern[dom],
                         "algorithmic_bytes_per_launch": samples_launch * ALGO_BYTES[dom],
                         "bytes_per_stereo_sample": ALGO_BYTES[dom], "traffic_source": traffic_src,
                         "kernels_ms_per_launch": kern, "kernels_ms_isolated": kern_iso,
                         "timing": "HIP events on each launch's stream while neighbouring chunks' "
                                   "kernels overlap (cross-chunk pipelining, as in the timed region)",
                         "gpu_ms_per_step_events": kern_ms,
                         "chain_gbs": value * sum(ALGO_BYTES[k] for k in kern) / 1e9},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
