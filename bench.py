#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: stereo samples/sec whole-node, full chain
(tonegen -> vibrato -> overdrive -> reverb -> whirl) at 48 kHz, 4096 organ instances
per GPU (configs[2] at N=1; configs[3] = 8 x 4096 at N=8, weak scaling), with
max|err| vs the CPU chain.

A "step" is one render call over the batch: every instance renders `--blocks`
128-sample blocks (default 2048 = 262144 stereo samples, 5.46 s of audio, per instance: one
steady chunk of the engine, i.e. one launch of each of the six stages).  Inputs are
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

# Algorithmic HBM bytes per stereo sample, per kernel.
# Only what the algorithm itself must move counts: the reverb's 13 delay lines x 2
# channels streamed once per cycle (8 B write + 8 B read, FP64) and the 8 B L/R output.
#   k_rv_core = the 12 network lines (A..L) x 2 ch x 16 B              = 384 B
#   k_rv_pre  = the predelay line M x 2 ch x 16 B                      =  32 B
#   k_whirl   = L/R float32 output                                     =   8 B
# The implementation's inter-stage streams (mid0/mid1/rvA/rvB/mid2) are NOT algorithmic; they
# show up in the PMC bytes instead.  Step total: 424 B (step_frac, the north_star's figure).
ALGO_BYTES = {"k_tonegen": 0, "k_mixpre": 0, "k_rv_pre": 32, "k_rv_core": 384, "k_rv_post": 0, "k_whirl": 8}
# Ceilings (/opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters and constants):
HBM_PEAK_GBS = 8000.0  # HBM3E 8.0 TB/s spec
CLOCK_GHZ = 2.4        # max clock
SIMDS = 256 * 4        # 256 CUs x 4 SIMD-32
# VALU issue cost of a wave64 instruction on a SIMD-32, in cycles: 2 for FP32 / integer;
# FP64 add / mul / fma at half the FP32 rate (78.6 vs 157.3 TFLOP/s): 4; an FP32
# transcendental (v_exp / v_sin / v_rcp ...) 2x a plain op: 4; an FP64 one: 16 (quarter of FP64)
VALU_CYC = {"base": 2.0, "f64": 4.0, "trans32": 4.0, "trans64": 16.0}
VALU_CYC_SOURCE = "spec-derived (78.6 vs 157.3 TFLOP/s)"
# measured on the box when available (tools/valu_calib.py: issue-bound probes of each
# instruction kind, cycles per wave64 instruction per SIMD), replacing the spec-derived costs
VALU_CALIB_JSON = ROOT / "profiles" / "valu_calib.json"
if VALU_CALIB_JSON.exists():
    try:
        _vc = json.loads(VALU_CALIB_JSON.read_text())["valu_cyc"]
        VALU_CYC = {k: round(float(_vc[k]), 2) for k in VALU_CYC}
        VALU_CYC_SOURCE = f"measured: {VALU_CALIB_JSON.relative_to(ROOT)} (tools/valu_calib.py)"
    except (KeyError, ValueError, TypeError):
        pass
VALU_PEAK_TOPS = SIMDS * CLOCK_GHZ * 1e9 / VALU_CYC["base"] * 64 / 1e12  # T lane-ops/s at the FP32 issue rate
# MI355X_MICROARCH.md, LDS/L2 gather table: rows shared by every workgroup of an XCD come
# from its L2 at 16.8-18.8 TB/s chip-wide (measured); the tonegen-only workload's wave-bank
# gathers are that pattern (one shared bank, every instance reading the same wheels)
L2_PEAK_GBS = 18800.0
PMC_JSON = ROOT / "profiles" / "kernel_pmc.json"  # written by tools/kernel_pmc.py


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096, help="instances per GPU")
    ap.add_argument("--blocks", type=int, default=2048,
                    help="128-sample blocks per step (one render call; a steady chunk is up to 2048 blocks)")
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
    ap.add_argument("--isolated", type=int, default=3,
                    help="steps timed with each kernel alone (pipelining off): the unloaded launch times "
                         "the per-kernel roofline divides by (0: skip)")
    ap.add_argument("--steady64", type=int, default=1,
                    help="steps also timed with 64-block chunks (tbf_set_steady_chunk(64)): the figure of a "
                         "workload with an event at least every 64 blocks, comparable with rounds 1-3")
    ap.add_argument("--pmc", default=str(PMC_JSON), help="per-kernel PMC profile (tools/kernel_pmc.py)")
    ap.add_argument("--kernel-steps", type=int, default=None,
                    help="extra steps timed per kernel with HIP events for the roofline (default = --steps)")
    ap.add_argument("--stage-check", type=int, default=1,
                    help="per-stage max|err| (tonegen / preamp / reverb taps) of the checked instances")
    ap.add_argument("--dry-run", type=int, default=0,
                    help="host-only engines (device -1), no render: exercises the rank setup, the sharding, "
                         "the max-over-ranks reductions and the JSON contract without a GPU")
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
    by oracle/Makefile with its release flags (oracle/_ref/fast/libtbfref.so; the strict
    build when that is absent), driven like synthSound; kind "port": the oracle's C
    restatement."""
    idx, blocks, sr, kind = args
    import scenarios as S
    from orc_bind import Chain, Template, load_oracle, load_ref
    lib = load_oracle()
    ref = load_ref(fast=True) if kind == "reference" else None
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


def host_info():
    """CPU model, glibc version, visible cores and the core lease of this process."""
    import platform
    model = None
    try:
        for ln in Path("/proc/cpuinfo").read_text().splitlines():
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        visible = len(os.sched_getaffinity(0))
    except AttributeError:
        visible = os.cpu_count() or 1
    lease = os.environ.get("OMP_NUM_THREADS")
    return {"cpu_model": model, "glibc": "-".join(platform.libc_ver()), "cores_visible": visible,
            "core_lease": int(lease) if lease and lease.isdigit() else None}


def cpu_baseline(n_inst, blocks, sr):
    import multiprocessing as mp
    from orc_bind import REF_FAST_SO, REF_SO
    kind = "reference" if (REF_FAST_SO.exists() or REF_SO.exists()) else "port"
    build = None
    if kind == "reference":
        build = ("-O3 -ffast-math -fno-finite-math-only (the reference's release flags, common.mak:16-18)"
                 if REF_FAST_SO.exists() else "-O2 -ffp-contract=off (strict build; release build absent)")
    hi = host_info()
    # every core this process may use: the GPU box leases a fixed share of the host per GPU
    # (OMP_NUM_THREADS there; nproc shows the whole machine), so that share is the pool
    cores = hi["core_lease"] or hi["cores_visible"]
    cores = max(1, min(cores, hi["cores_visible"], n_inst))
    parts = [list(range(k, n_inst, cores)) for k in range(cores)]
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(cores) as pool:
        res = pool.map(_cpu_worker, [(p, blocks, sr, kind) for p in parts])
    wall = time.perf_counter() - t0
    samples = sum(r[0] for r in res)
    busy = max(r[1] for r in res)  # render time of the slowest worker (construction excluded)
    what = ("the reference's src/tonegen.cpp, vibrato.cpp, overdrive.cpp, reverb.cpp, whirl.cpp "
            f"compiled by oracle/Makefile, {build}" if kind == "reference" else "oracle/ C restatement")
    return {"value": samples / busy, "unit": "stereo samples/s", "cores": cores, "kind": kind,
            "sample": f"{n_inst} instances x {blocks} blocks ({blocks * 128 / sr:.2f} s audio each), "
                      f"{what}, {cores} worker processes (one per leased core), construction excluded "
                      f"(wall {wall:.1f}s)", **hi}


def oracle_run(wl, g, total_blocks, last_blocks):
    """The oracle's L, R and stage taps (tonegen, preamp, reverb) of instance g over the
    last `last_blocks` of `total_blocks`."""
    from orc_bind import Chain, Template, load_oracle
    lib = load_oracle()
    j = wl.tuning_of(g)
    tpl = Template(lib, sr=wl.sr, mts128=wl.mts[wl.names[j]], seed=wl.tpl_seed(j))
    ch = Chain(lib, tpl, wl.seed_of(g))
    if wl.kind == "cfg2":
        ch.chain(1)
    for (_, kind, a, v) in wl.scenario(g):
        (ch.note if kind == "note" else ch.param)(a, v)
    ch.render(total_blocks - last_blocks)
    return ch.render(last_blocks, stages=True)


def _err(x, y):
    import numpy as np
    d = np.abs(x.astype(np.float64) - y.astype(np.float64))
    return float(d.max()) if d.size else 0.0, int(np.sum(x.view(np.uint32) == y.view(np.uint32))), x.size


def stage_taps(T, wl, first, n_check, total_blocks, last_blocks, device):
    """The GPU's tonegen / preamp / reverb stage outputs of the checked instances: small
    engines in the parity-tap chain modes (TBF_CHAIN_TONEGEN / _TAP_PREAMP / _TAP_REVERB)
    replaying the same instances and script for the same number of blocks."""
    import numpy as np
    taps = {}
    for mode, name in ((1, "tonegen"), (2, "preamp"), (3, "reverb")):
        if wl.kind == "cfg2" and mode > 1:
            continue
        eng = T.Engine(sample_rate=wl.sr, device=device, chain=mode)
        setup_instances(eng, wl, first, n_check)
        # the same render calls as the timed engine: whole steps of last_blocks blocks
        parts = []
        left = total_blocks
        while left:
            nb = min(left, last_blocks)
            L, _ = eng.render(nb)
            parts = (parts + [L])[-2:]
            left -= nb
        L = np.concatenate(parts, axis=1) if parts else np.zeros((n_check, 0), np.float32)
        taps[name] = L[:, -last_blocks * 128:]
        eng.close()
    return taps


def oracle_check(wl, rank_first, n_check, total_blocks, last_blocks, gpu_L, gpu_R, taps=None):
    """max|err| and bit-exact fraction of the last step's outputs vs the CPU oracle for
    the first instances of this rank, and per stage when the GPU stage taps are given."""
    stages = {"whirl_L": [0.0, 0, 0], "whirl_R": [0.0, 0, 0]}
    for i in range(n_check):
        L, R, A, B, C = oracle_run(wl, rank_first + i, total_blocks, last_blocks)
        pairs = [("whirl_L", gpu_L[i], L), ("whirl_R", gpu_R[i], R)]
        if taps:
            ref = {"tonegen": A, "preamp": B, "reverb": C}
            pairs += [(k, taps[k][i], ref[k]) for k in taps]
        for k, x, y in pairs:
            e, ex, n = _err(x, y)
            acc = stages.setdefault(k, [0.0, 0, 0])
            acc[0] = max(acc[0], e)
            acc[1] += ex
            acc[2] += n
    out = {k: {"max_err": v[0], "bit_exact_frac": v[1] / max(v[2], 1)} for k, v in stages.items()}
    err = max(out["whirl_L"]["max_err"], out["whirl_R"]["max_err"])
    exact = (stages["whirl_L"][1] + stages["whirl_R"][1]) / max(stages["whirl_L"][2] + stages["whirl_R"][2], 1)
    return err, exact, out


def lib_hash():
    import hashlib
    import tunebfree_amd as T
    return hashlib.sha256(Path(T.LIB_PATH).read_bytes()).hexdigest()[:16]


def kernel_bounds(ms, pmc, scale=1.0):
    """One kernel against its two ceilings, from its unloaded launch time (ms) and its PMC
    counts per launch (tools/kernel_pmc.py), scaled by `scale` from the profiled launch's
    samples to the timed launch's: HBM bytes / time against 8 TB/s, and VALU issue cycles
    (instruction counts x their SIMD-32 issue cost) / time against every SIMD issuing at
    2.4 GHz.  Both fractions are of the whole chip."""
    c = {k: v * scale for k, v in pmc["counters"].items()}
    row = {"kernel": pmc.get("kernel"), "ms_isolated": ms, "pmc_ms": pmc.get("pmc_ms")}
    sec = ms * 1e-3
    if "hbm_bytes" in pmc:
        row["hbm_bytes"] = pmc["hbm_bytes"] * scale
        row["hbm_bytes_per_stereo_sample"] = pmc.get("hbm_bytes_per_stereo_sample")
        row["hbm_gbs"] = row["hbm_bytes"] / sec / 1e9
        row["hbm_frac"] = row["hbm_gbs"] / HBM_PEAK_GBS
    if "SQ_INSTS_VALU" in c:
        f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64"))
        t32, t64 = c.get("SQ_INSTS_VALU_TRANS_F32", 0.0), c.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
        cyc = (VALU_CYC["base"] * c["SQ_INSTS_VALU"] + (VALU_CYC["f64"] - VALU_CYC["base"]) * f64
               + (VALU_CYC["trans32"] - VALU_CYC["base"]) * t32 + (VALU_CYC["trans64"] - VALU_CYC["base"]) * t64)
        row["valu_insts"] = c["SQ_INSTS_VALU"]
        row["valu_issue_cycles"] = cyc
        row["valu_tops"] = cyc / VALU_CYC["base"] * 64 / sec / 1e12
        row["valu_frac"] = cyc / (SIMDS * CLOCK_GHZ * 1e9 * sec)
    if c.get("SQ_WAVE_CYCLES"):
        if "SQ_WAIT_ANY" in c:
            row["wait_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]  # waves parked (waitcnt / barrier)
    if c.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in c:
        row["lane_util"] = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
    if "clock_ghz" in pmc:
        row["clock_ghz_profiled"] = pmc["clock_ghz"]
    fr = {k: row[k + "_frac"] for k in ("hbm", "valu") if k + "_frac" in row}
    row["bound"] = max(fr, key=fr.get) if fr else None
    return row


def roofline(a, B, nsamp, elapsed, samples_launch, launches, algo, kern, kern_iso, bank_entries):
    """The bench line's roofline object: every kernel against the ceiling that binds it
    (unloaded launch time, PMC bytes and VALU issue of the same build); the dominant kernel
    (longest unloaded launch) in the top-level fields; the north_star's step-level HBM
    fraction of the 424-B byte model beside it."""
    pmc, pmc_note = None, None
    if Path(a.pmc).exists():
        pj = json.loads(Path(a.pmc).read_text())
        wl = {"batch": B, "blocks": a.blocks, "sr": a.sr, "chain": a.chain}
        if pj.get("workload") != wl:
            pmc_note = f"{a.pmc}: another workload ({pj.get('workload')})"
        else:
            pmc = pj
            if pj.get("build") != lib_hash():
                pmc_note = f"{a.pmc}: profiled on build {pj.get('build')}, this library is {lib_hash()}"
    step_bytes = sum(algo[k] for k in kern)
    step_gbs = B * nsamp * step_bytes / (elapsed / a.steps) / 1e9  # per GPU
    times = kern_iso or kern
    rows = {}
    for k, ms in times.items():
        if pmc and k in pmc["kernels"]:
            rows[k] = kernel_bounds(ms, pmc["kernels"][k], samples_launch / pmc["samples_per_launch"])
        else:
            rows[k] = {"ms_isolated": ms if kern_iso else None}
        rows[k]["ms_as_rendered"] = kern.get(k)
        rows[k]["algorithmic_bytes_per_stereo_sample"] = algo.get(k, 0)
    dom = max(times, key=times.get)
    d = rows[dom]
    roof = {"kernel": dom, "kernel_ms_isolated": times[dom] if kern_iso else None,
            "bound": d.get("bound"), "achieved": None, "peak": None, "unit": None, "frac": None,
            "traffic": d.get("hbm_bytes"),
            "hbm_frac": d.get("hbm_frac"), "valu_frac": d.get("valu_frac"),
            # the 424-B model's bytes for this kernel's launch (no fraction: k_rv_core_lds keeps its
            # 384 B per sample of line traffic in LDS, so they would read above the HBM peak)
            "algorithmic_bytes_per_launch": samples_launch * algo.get(dom, 0),
            "launches_per_step": launches,
            "step_bytes_per_stereo_sample": step_bytes, "step_gbs_per_gpu": step_gbs,
            "step_frac": step_gbs / HBM_PEAK_GBS,
            "kernels": rows,
            "pmc_source": (pmc or {}).get("source"), "pmc_build": (pmc or {}).get("build"),
            "pmc_build_match": bool(pmc) and pmc.get("build") == lib_hash(), "pmc_note": pmc_note,
            "valu_issue_cycles": VALU_CYC, "valu_issue_cycles_source": VALU_CYC_SOURCE,
            "method": "each kernel's unloaded launch time (every kernel alone, pipelining off, HIP events on "
                      "its stream) against its own ceilings: HBM = PMC FETCH_SIZE x 2 + WRITE_SIZE bytes per "
                      "launch / time vs 8 TB/s; VALU = SQ_INSTS_VALU (+ FP64 / transcendental issue cost) x "
                      "cycles (valu_issue_cycles) / time vs 1024 SIMDs at 2.4 GHz; bound = the larger; the dominant "
                      "kernel = the longest unloaded launch"}
    if d.get("bound") == "hbm":
        roof.update({"achieved": d["hbm_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": d["hbm_frac"]})
    elif d.get("bound") == "valu":
        roof.update({"achieved": d["valu_tops"], "peak": VALU_PEAK_TOPS, "unit": "T lane-ops/s (FP32-rate)",
                     "frac": d["valu_frac"]})
    if bank_entries is not None and "k_tonegen" in times:
        # tonegen only (configs[1]) is L2-bound: every program entry of a
        # block gathers one wheel's 128 samples from the shared bank, 4 B per entry and sample
        l2b = 4.0 * bank_entries
        l2a = samples_launch * l2b / (times["k_tonegen"] * 1e-3) / 1e9
        roof["l2"] = {"kernel": "k_tonegen", "achieved": l2a, "peak": L2_PEAK_GBS, "unit": "GB/s",
                      "frac": l2a / L2_PEAK_GBS, "bytes_per_stereo_sample": l2b,
                      "bank_entries_per_block": bank_entries,
                      "note": "tonegen only: the wave-bank gathers, 4 B x program entries per sample, from the "
                              "shared L2-resident bank; HBM moves only the 8 B output"}
    return roof


def launch_ranks(n):
    """`bench.py --gpus N` with no launcher around it: start N ranks under
    torch.distributed.run as a CHILD process (this process has not touched HIP: nothing
    above imports torch.cuda or the engine), relay its output (rank 0's JSON line) and
    return its exit code.  One rank per GPU; TBF_BENCH_ONE_DEVICE=1 puts every rank on
    device 0 (the rehearsal on a one-GPU lease)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", str(ROOT / "bench.py")] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env, cwd=str(ROOT)).returncode


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world} (launch one rank per GPU, or drop the "
              f"launcher and let bench.py start the ranks itself)", file=sys.stderr)
        sys.exit(2)
    import numpy as np
    import torch
    from tunebfree_amd.shard import shard
    dist = None
    if world > 1:
        # the only cross-rank traffic is the barrier and three scalars (elapsed, max|err|,
        # dry-run checksum): gloo on the host, no RCCL (the data path has no collective)
        import torch.distributed as dist
        dist.init_process_group("gloo")
    if not a.dry_run:
        one_dev = os.environ.get("TBF_BENCH_ONE_DEVICE", "0") == "1"
        ndev = torch.cuda.device_count()  # counts devices without initialising HIP on this image
        if world > 1 and not one_dev and local >= ndev:
            print(f"bench.py: rank {rank} (local {local}) has no GPU: {ndev} visible for {world} ranks "
                  f"(TBF_BENCH_ONE_DEVICE=1 shares device 0 for a rehearsal)", file=sys.stderr)
            sys.exit(2)
        torch.cuda.set_device(0 if (world == 1 or one_dev) else local)
    import tunebfree_amd as T

    # weak scaling: --batch instances per GPU, world * batch in all, contiguous shards
    first_global, B = shard(a.batch * world, rank, world)
    if a.sr is None:
        a.sr = 96000.0 if a.workload == "cfg5" else 48000.0
    wl = Workload(a.workload, a.sr)
    if a.workload == "cfg2":
        a.chain = 1  # TBF_CHAIN_TONEGEN
    device = -1 if a.dry_run else torch.cuda.current_device()
    eng = T.Engine(sample_rate=a.sr, device=device, chain=a.chain)
    setup_instances(eng, wl, first_global, B)
    nsamp = a.blocks * 128

    def reduce(x, op="max"):
        if not dist:
            return float(x)
        t = torch.tensor([float(x)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
        return float(t.item())

    def sync():
        if not a.dry_run:
            torch.cuda.synchronize()

    if a.dry_run:
        # no device: the "step" is the host control step a render makes per block for every
        # instance of the shard (tbf_debug_render_program), so the contract runs end to end
        import ctypes as C
        lib = T.load_library()
        fn = lib.tbf_debug_render_program
        fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]
        buf = np.zeros(9 * 600, np.float32)
        chk = [0]

        def step():  # exact integer checksum of every instance's program (order-independent)
            for i in range(B):
                n = fn(eng._h, i, buf.ctypes.data, 600)
                chk[0] += int(buf[: 9 * n].view(np.uint32).astype(np.int64).sum()) * (first_global + i + 1)
    else:
        outL = torch.empty((B, nsamp), dtype=torch.float32, device="cuda")
        outR = torch.empty((B, nsamp), dtype=torch.float32, device="cuda")
        stream = torch.cuda.Stream()  # a real stream: the kernel and the timing events share it
        torch.cuda.set_stream(stream)
        sptr = stream.cuda_stream

        def step():
            eng.render_device(a.blocks, outL.data_ptr(), outR.data_ptr(), nsamp, sptr)

    for _ in range(a.warmup):
        step()
    sync()
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(a.steps):
        step()
    sync()
    if dist:
        dist.barrier()
    sync()
    elapsed = reduce(time.perf_counter() - t0)
    total_samples = world * a.batch * nsamp * a.steps  # every rank's instances (shard sums to world * batch)
    value = total_samples / elapsed

    kern, kern_iso, max_err, exact, per_stage, steady64 = {}, None, None, None, None, None
    # launch sets per step: the timed steps have no control deltas, so each chunk is up to the
    # engine's steady chunk (TBF_STEADY_CHUNK, default TBF_STEADY_DEFAULT = 512 blocks; 64 with deltas)
    chunk = eng.chunks()[1] if not a.dry_run else 64
    launches = -(-a.blocks // chunk)
    ksteps = a.steps if a.kernel_steps is None else a.kernel_steps
    if not a.dry_run:
        # per-kernel launch durations (HIP events on each launch's stream, inside the
        # engine), rendered exactly like the timed region (cross-chunk pipelining on, so a
        # duration includes the overlap with the neighbouring chunk's kernels); a separate
        # pass so the events do not perturb the timed region above
        eng.kernel_times(True)
        for _ in range(ksteps):
            step()
        torch.cuda.synchronize()
        kt = eng.kernel_times()
        eng.kernel_times(False)
        kern = {k: v[0] / v[1] for k, v in kt.items() if v[1]}
        extra_blocks = ksteps * a.blocks
        if a.isolated:  # each kernel alone on the GPU (pipelining off): the unloaded launch times
            eng.kernel_times("serial")
            for _ in range(a.isolated):
                step()
            torch.cuda.synchronize()
            kt = eng.kernel_times()
            eng.kernel_times(False)
            kern_iso = {k: v[0] / v[1] for k, v in kt.items() if v[1]}
            extra_blocks += a.isolated * a.blocks
        if a.steady64 and a.blocks > 64:
            # the same steps in 64-block chunks (every launch 64 blocks, as a workload with an
            # event at least every 64 blocks renders): one warmup step, then a.steady64 timed
            chunk0 = eng.chunks()[1]
            eng.set_steady_chunk(64)
            step()
            sync()
            t64 = time.perf_counter()
            for _ in range(a.steady64):
                step()
            sync()
            t64 = time.perf_counter() - t64
            eng.set_steady_chunk(chunk0)
            steady64 = {"ms_per_64_blocks": t64 / a.steady64 / (a.blocks / 64) * 1e3,
                        "value": B * nsamp * a.steady64 / t64, "steps": a.steady64,
                        "note": "rank-local: the same render with every chunk 64 blocks long "
                                "(tbf_set_steady_chunk(64); rounds 1-3 measured this step)"}
            extra_blocks += (1 + a.steady64) * a.blocks
        # parity on the last step (first --check instances of this rank), per stage
        total_blocks = (a.warmup + a.steps) * a.blocks + extra_blocks
        if a.check:
            gL = outL[: a.check].cpu().numpy()
            gR = outR[: a.check].cpu().numpy()
            taps = stage_taps(T, wl, first_global, a.check, total_blocks, a.blocks, device) if a.stage_check else None
            max_err, exact, per_stage = oracle_check(wl, first_global, a.check, total_blocks, a.blocks, gL, gR, taps)
    dry_sum = reduce(chk[0] % (1 << 50), "sum") if a.dry_run else None
    max_err = reduce(max_err or 0.0) if (a.check and not a.dry_run) else None

    bank_entries = None
    if a.chain == 1 and not a.dry_run:
        # tonegen only (configs[1]) is L2-bound: every program entry of a
        # block gathers one wheel's 128 samples from the shared bank, 4 B per entry and
        # sample.  Entries per block: the device programs of up to 32 instances.
        import ctypes as C
        fn = T.load_library().tbf_debug_device_program
        fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]
        pbuf = np.zeros(9 * 600, np.float32)
        cnt = [fn(eng._h, i, pbuf.ctypes.data, 600) for i in range(0, B, max(1, B // 32))]
        bank_entries = float(np.mean([c for c in cnt if c >= 0])) if cnt else None

    if rank == 0:
        samples_launch = B * min(a.blocks, chunk) * 128  # stereo samples one launch of a stage renders
        algo = dict(ALGO_BYTES)
        if a.chain == 1:  # tonegen only: k_mixpre writes L and R (8 B); bank reads are L2-resident
            algo["k_mixpre"] = 8
        roof = roofline(a, B, nsamp, elapsed, samples_launch, launches, algo, kern, kern_iso, bank_entries) \
            if kern else None
        cpu = cpu_baseline(a.cpu_instances, a.cpu_blocks, a.sr) \
            if (a.cpu_baseline and world == 1 and a.workload == "cfg3" and not a.dry_run) else None
        line = {
            "metric": "stereo samples/sec whole-node, batch=4096 full chain @48kHz; max|err| vs CPU",
            "value": value, "unit": "stereo samples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32 (f64 reverb/overdrive)", "data": "synthetic",
            "config": {"workload": wl.describe(a.batch, world, a.blocks),
                       "batch_per_gpu": a.batch, "blocks_per_step": a.blocks, "sample_rate": a.sr,
                       "parallelism": f"instance-sharded x{world} (no collective)"},
            "max_err": max_err, "bit_exact_frac": exact, "checked_instances": a.check,
            "max_err_per_stage": per_stage,
            "roofline": roof,
            "steady64": steady64,
            "cpu_baseline": cpu,
        }
        if a.dry_run:
            line["dry_run"] = {"note": "host-only engines, no render: value/ms_per_step time one host "
                                       "control step per instance and step, not the DSP chain",
                               "shard_rank0": [first_global, B],
                               "checksum": dry_sum}  # sum over ranks of per-instance program checksums
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
