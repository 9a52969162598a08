"""GPU parity: the HIP render path (through the C-ABI) against the CPU oracle.

Gate (BASELINE.json north_star): max|err| <= 1e-5 per float32 sample vs the CPU
chain.  The float32 stages are computed in the reference's literal operation order,
so the expected outcome is bit-identity; the only licensed source of difference is
FP64 libm (GPU sin/asin vs glibc), reported as the bit-exact fraction.
"""
import numpy as np
import pytest

import scenarios as S
from enginerun import compare, engine_run, oracle_run

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _engine(chain=0, sr=48000.0, debug_flags=0):
    import tunebfree_amd as T
    return T.Engine(sample_rate=sr, device=0, chain=chain, debug_flags=debug_flags)


def _setup(oracle, n, scen_fn, chain=0, tpl_seed=7, sr=48000.0, debug_flags=0, cfg=None):
    from orc_bind import Cfg, Template
    eng = _engine(chain, sr, debug_flags)
    if cfg is not None:  # as a cfg file's text, through tbf_config_parse
        items = list(cfg.items()) if isinstance(cfg, dict) else list(cfg)
        assert eng.config_parse("# cfg\n" + "".join(f"{k} = {v}\n" for k, v in items)) == len(items)
    tid = eng.template(seed=tpl_seed)
    seeds = [1000 + 17 * i for i in range(n)]
    eng.add_instances([tid] * n, seeds)
    tpl = Template(oracle, sr=sr, seed=tpl_seed, cfg=None if cfg is None else Cfg(oracle, cfg))
    scens = [scen_fn(i) for i in range(n)]
    return eng, tpl, seeds, scens


def test_gpu_tonegen_only_bitexact(oracle):
    eng, tpl, seeds, scens = _setup(oracle, 8, lambda i: S.bench_scenario(i, full=False), chain=1)
    L, R = engine_run(eng, scens, 24)
    oL, oR, oA, _, _ = oracle_run(oracle, tpl, seeds, scens, 24, chain=1)
    err, exact = compare(L, oA)
    print(f"tonegen max|err|={err:.3g} bit-exact={exact:.6f}")
    assert err == 0.0 and exact == 1.0
    assert np.array_equal(L, R)


def test_gpu_tonegen_block_ranges(oracle):
    """A chunk without control deltas may split each instance's blocks over several waves
    (tbf_launch.tgSplit): a range after the first starts one warm-up block early from the
    chunk-start state advanced in closed form.  Tonegen-only and full chain, chunks of 64
    and 40 blocks after an event block, vibrato and percussion routed (and, tonegen only,
    without percussion: the gain chases settle at a fixed point and k_tonegen writes the
    products itself): the default split, ranges of one block's granularity
    (TBF_TG_SPLIT=5) and no split (TBF_TG_SPLIT=1) are bit-identical, and match the
    oracle."""
    import os
    for chain, full in ((1, True), (1, False), (0, True)):
        outs = []
        for env in ({}, {"TBF_TG_SPLIT": "5"}, {"TBF_TG_SPLIT": "1"}):
            os.environ.update(env)
            try:
                eng, tpl, seeds, scens = _setup(oracle, 40, lambda i: S.bench_scenario(i, full=full), chain=chain)
            finally:
                for k in env:
                    os.environ.pop(k, None)
            parts = [engine_run(eng, scens, 1), eng.render(64), eng.render(40)]
            eng.close()
            outs.append((np.concatenate([p[0] for p in parts], axis=1), np.concatenate([p[1] for p in parts], axis=1)))
        pick = [0, 13, 39]
        res = oracle_run(oracle, tpl, [seeds[i] for i in pick], [scens[i] for i in pick], 105, chain=chain)
        ref = res[2] if chain == 1 else res[0]
        err, exact = compare(outs[0][0][pick], ref)
        print(f"chain {chain} (Jazz-1 {full}): max|err|={err:.3g} bit-exact={exact:.6f}")
        assert err <= TOL
        for o in outs[1:]:
            assert all(np.array_equal(a.view(np.uint32), b.view(np.uint32)) for a, b in zip(outs[0], o))


@pytest.mark.parametrize("tap,idx", [(2, 3), (3, 4)])
def test_gpu_stage_taps(oracle, tap, idx):
    eng, tpl, seeds, scens = _setup(oracle, 6, S.bench_scenario, chain=tap)
    L, _ = engine_run(eng, scens, 32)
    ref = oracle_run(oracle, tpl, seeds, scens, 32)[idx]
    err, exact = compare(L, ref)
    print(f"tap {tap}: max|err|={err:.3g} bit-exact={exact:.6f}")
    assert err <= TOL


def test_gpu_full_chain_bench(oracle):
    eng, tpl, seeds, scens = _setup(oracle, 8, S.bench_scenario)
    L, R = engine_run(eng, scens, 64)
    oL, oR, *_ = oracle_run(oracle, tpl, seeds, scens, 64)
    eL, xL = compare(L, oL)
    eR, xR = compare(R, oR)
    print(f"full chain: max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL


def test_gpu_full_chain_odd_batch_mixed_scenarios(oracle):
    """k_rv_pre and k_rv_post serve 32 instances per workgroup (a chain per lane): a batch
    of 37 leaves the second workgroup with 5, and neighbouring instances with different
    scripts (events, quiet ones, reverb-heavy) must not leak into each other."""
    def scen(i):
        if i in (2, 33):
            return []  # silent instances between playing ones
        return S.event_scenario(i) if i % 2 else S.bench_scenario(i)
    eng, tpl, seeds, scens = _setup(oracle, 37, scen)
    L, R = engine_run(eng, scens, 40)
    oL, oR, *_ = oracle_run(oracle, tpl, seeds, scens, 40)
    eL, xL = compare(L, oL)
    eR, xR = compare(R, oR)
    print(f"odd batch: max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL
    assert float(np.abs(L[1]).max()) > 1e-3 and float(np.abs(L[3]).max()) > 1e-3


def test_gpu_full_chain_events(oracle):
    eng, tpl, seeds, scens = _setup(oracle, 6, S.event_scenario)
    L, R = engine_run(eng, scens, 72)
    oL, oR, *_ = oracle_run(oracle, tpl, seeds, scens, 72)
    eL, xL = compare(L, oL)
    eR, xR = compare(R, oR)
    print(f"events: max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL


@pytest.mark.parametrize("debug_flags", [0, 1])
def test_gpu_vs_committed_reference_vectors(debug_flags):
    """The HIP engine against the reference's own compiled chain (committed vectors,
    tests/golden/ref_vectors.npz): 44.1/48/96 kHz (whirl ring W=512/1024), 12-TET /
    19-TET / p4 / bagpipe4 / duodene / 5TET templates, event scripts, config-5 random
    drawbars, the parameter sweep (overdrive character, reverb mix, percussion variants,
    clusters, pedal keys, rotary stop <-> fast).  debug_flags=1 (TBF_DEBUG_FORCE_SERIAL)
    runs every guarded stage on its serial replay instead of the lane-parallel fast
    path: both must match."""
    import json
    from pathlib import Path
    import tunebfree_amd as T
    from golden.make_ref_vectors import scenario
    gold = Path(__file__).resolve().parent / "golden"
    z = np.load(gold / "ref_vectors.npz")
    tunings = json.loads((gold / "tunings.json").read_text())
    worst = 0.0
    for c in json.loads(str(z["cases"])):
        eng = T.Engine(sample_rate=c["sr"], device=0, chain=c["chain"], debug_flags=debug_flags)
        m = None if c["tuning"] is None else np.array(tunings[c["tuning"]], np.float64)
        tid = eng.template(mts128=m, seed=c["tpl_seed"])
        eng.add_instances([tid], [c["inst_seed"]])
        L, R = engine_run(eng, [scenario(*c["scenario"])], c["nblocks"])
        for got, k in ((L[0], "L"), (R[0], "R")):
            err, exact = compare(got, z[f"{c['name']}/{k}"])
            print(f"{c['name']}/{k}: max|err|={err:.3g} bit-exact={exact:.6f}")
            worst = max(worst, err)
        flags = eng.error_flags()
        print(f"{c['name']}: paths taken 0x{flags:x}")
        if debug_flags and c["chain"] == 0:
            assert flags & (T.engine.PATH_WH_ANGLE | T.engine.PATH_WH_MOTION | T.engine.PATH_RV_PHASE) == \
                T.engine.PATH_WH_ANGLE | T.engine.PATH_WH_MOTION | T.engine.PATH_RV_PHASE, hex(flags)
        eng.close()
    assert worst <= TOL


def test_gpu_config5_mixed_tunings_96k(oracle):
    """BASELINE config 5 shape at test size: 96 kHz, one shared template per tuning
    (7 tunings of the reference's tests), per-instance random drawbars, several
    templates interleaved inside one launch."""
    import json
    from pathlib import Path
    import tunebfree_amd as T
    from orc_bind import Template
    tunings = json.loads((Path(__file__).resolve().parent / "golden" / "tunings.json").read_text())
    names = sorted(tunings, key=lambda k: (tunings[k] is not None, k))
    eng = T.Engine(sample_rate=96000.0, device=0)
    tids, tpls = {}, {}
    for j, nm in enumerate(names):
        m = None if tunings[nm] is None else np.array(tunings[nm], np.float64)
        tids[nm] = eng.template(mts128=m, seed=100 + j)
        tpls[nm] = Template(oracle, sr=96000.0, mts128=m, seed=100 + j)
    n = 2 * len(names)
    pick = [names[(5 * i) % len(names)] for i in range(n)]
    seeds = [7000 + i for i in range(n)]
    eng.add_instances([tids[p] for p in pick], seeds)
    scens = [S.random_drawbar_scenario(i) for i in range(n)]
    L, R = engine_run(eng, scens, 24)
    worst, ex = 0.0, []
    for i in range(n):
        oL, oR, *_ = oracle_run(oracle, tpls[pick[i]], [seeds[i]], [scens[i]], 24)
        for a, b in ((L[i], oL[0]), (R[i], oR[0])):
            e, x = compare(a, b)
            worst = max(worst, e)
            ex.append(x)
    print(f"config5: {n} instances, {len(names)} tunings, max|err|={worst:.3g} bit-exact={min(ex):.6f}")
    assert worst <= TOL


def test_gpu_program_install_matches_clap_script(oracle):
    """§8(f) row 4: an organ configured by installProgram ("Jazz 1 all" in .pgm syntax,
    src/program.cpp:735-921) plus the character knob renders bit-identically to the
    oracle driven by the CLAP parameter script of the bench scenario."""
    from test_control_cpu import PGM
    eng, tpl, seeds, scens = _setup(oracle, 4, S.bench_scenario)
    assert eng.program_parse(PGM) == 4
    script = []
    for i in range(4):
        eng.program_install(i, 0)
        eng.set_param(i, S.P_CHARACTER, 0.5)
        script.append([(0, "note", k, 1) for k in S.chord_for(i)])
    L, R = engine_run(eng, script, 40)
    oL, oR, *_ = oracle_run(oracle, tpl, seeds, scens, 40)
    eL, xL = compare(L, oL)
    eR, xR = compare(R, oR)
    print(f"program install: max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL


def _script_events(eng, scens):
    rows = []
    for i, sc in enumerate(scens):
        for (b, kind, a, v) in sc:
            if kind == "note":
                rows.append((b, i, 0, a, 1.0 if v else 0.0))
            else:
                rows.append((b, i, 1, a, float(v)))
    return eng.events(rows)


def test_gpu_render_events_one_call(oracle):
    """§8(f) row 1: the event script of every instance (chord changes, drawbar, rotary,
    percussion, vibrato and swell events at blocks 0/32/40/48/56) in ONE
    tbf_render_events call -- per-block control deltas instead of launch segments --
    is bit-identical to the oracle."""
    import torch
    eng, tpl, seeds, scens = _setup(oracle, 6, S.event_scenario)
    nb = 72
    L = torch.zeros((6, nb * 128), dtype=torch.float32, device="cuda")
    R = torch.zeros_like(L)
    eng.render_events_device(nb, _script_events(eng, scens), L.data_ptr(), R.data_ptr(), nb * 128)
    eng.synchronize()
    oL, oR, *_ = oracle_run(oracle, tpl, seeds, scens, nb)
    eL, xL = compare(L.cpu().numpy(), oL)
    eR, xR = compare(R.cpu().numpy(), oR)
    print(f"render_events: max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL


def test_gpu_render_events_dense_across_chunks(oracle):
    """Events on many blocks and across the 64-block chunk boundary (notes every 7
    blocks, MIDI control functions, a programme change, whirl bypass toggles), split
    over two calls."""
    import torch
    from test_control_cpu import PGM
    eng, tpl, seeds, scens = _setup(oracle, 3, S.bench_scenario)
    assert eng.program_parse(PGM) == 4
    cid = eng.control_id("upper.drawbar4")
    assert cid >= 0 and eng.control_id("nope") < 0
    rows, oscen = [], []
    for i in range(3):
        sc = list(scens[i])
        for b in range(5, 150, 7):
            k = 60 + (b + 3 * i) % 12
            sc.append((b, "note", k, 1))
            sc.append((b + 3, "note", k, 0))
        sc.append((63, "param", S.P_DRAWBAR + 3, 5))   # same effect as upper.drawbar4 <- CC 48
        sc.append((64, "param", S.P_HORN, 2))
        # whirl bypass on/off mid-chunk and across the chunk edge (horn filter A runs
        # a sub-block ahead; it must not run into a bypassed block)
        for (b, v) in ((30, 1), (33, 0), (63, 1), (64, 0), (99, 1), (101, 0)):
            sc.append((b, "param", S.P_WHIRL_BYPASS, v))
        oscen.append(sc)
        for (b, kind, a, v) in sc:
            if (b, a) == (63, S.P_DRAWBAR + 3):
                rows.append((b, i, 2, cid, 48.0))  # rint ((127 - 48) * 8 / 127) = 5
            elif kind == "note":
                rows.append((b, i, 0, a, 1.0 if v else 0.0))
            else:
                rows.append((b, i, 1, a, float(v)))
    ev = eng.events(rows)
    nb = 160
    L = torch.zeros((3, nb * 128), dtype=torch.float32, device="cuda")
    R = torch.zeros_like(L)
    first = ev[ev["block"] < 100]
    rest = ev[ev["block"] >= 100].copy()
    rest["block"] -= 100
    eng.render_events_device(100, first, L.data_ptr(), R.data_ptr(), nb * 128)
    eng.render_events_device(60, rest, L[:, 100 * 128:].data_ptr(), R[:, 100 * 128:].data_ptr(), nb * 128)
    eng.synchronize()
    oL, oR, *_ = oracle_run(oracle, tpl, seeds, oscen, nb)
    eL, xL = compare(L.cpu().numpy(), oL)
    eR, xR = compare(R.cpu().numpy(), oR)
    print(f"dense events: max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL


def test_gpu_dense_events_threaded_host_control(oracle):
    """§8(f) row 1 at scale: 1200 instances with events on every block (a key released
    and one pressed, a drawbar move, a control function every 5 blocks) over 80 blocks
    (across the chunk edge).  With this many active instances the host front end steps
    on worker threads by instance range (stepChunkParallel); the output must equal, bit
    for bit, an engine stepping serially (TBF_HOST_SERIAL=1) for every instance, and the
    oracle for a sample of instances."""
    import os
    import torch
    import tunebfree_amd as T
    from orc_bind import Template
    n, nb = 1200, 80
    seeds = [3000 + i for i in range(n)]
    cid = None
    rows, oscen = [], [[] for _ in range(n)]
    for i in range(n):
        for (k, a, v) in S.jazz1_params():
            rows.append((0, i, 1, a, float(v)))
            oscen[i].append((0, k, a, v))
        for k in S.chord_for(i):
            rows.append((0, i, 0, k, 1.0))
            oscen[i].append((0, "note", k, 1))
        for b in range(1, nb):
            k0, k1 = 72 + (i + b - 1) % 12, 72 + (i + b) % 12
            rows.append((b, i, 0, k0, 0.0))
            oscen[i].append((b, "note", k0, 0))
            rows.append((b, i, 0, k1, 1.0))
            oscen[i].append((b, "note", k1, 1))
            rows.append((b, i, 1, S.P_DRAWBAR + 4, float((i + b) % 9)))
            oscen[i].append((b, "param", S.P_DRAWBAR + 4, (i + b) % 9))
    outs = []
    for serial in (False, True):
        if serial:
            os.environ["TBF_HOST_SERIAL"] = "1"
        try:
            eng = T.Engine(sample_rate=48000.0, device=0)
        finally:
            os.environ.pop("TBF_HOST_SERIAL", None)
        tid = eng.template(seed=7)
        eng.add_instances([tid] * n, seeds)
        cid = eng.control_id("upper.drawbar4")
        extra = [(b, i, 2, cid, float((7 * i + b) % 128)) for i in range(0, n, 3) for b in range(2, nb, 5)]
        ev = eng.events(rows + extra)
        L = torch.zeros((n, nb * 128), dtype=torch.float32, device="cuda")
        R = torch.zeros_like(L)
        eng.render_events_device(nb, ev, L.data_ptr(), R.data_ptr(), nb * 128)
        eng.synchronize()
        ht, _ = eng.host_time()
        outs.append((L.cpu().numpy(), R.cpu().numpy()))
        print(f"{'serial' if serial else 'threaded'} host control: {ht:.1f} ms")
        eng.close()
        del L, R
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1].view(np.uint32), outs[1][1].view(np.uint32))
    # the control-function events: upper.drawbar4 <- CC v is setDrawBar (3, rint ((127 - v) * 8 / 127))
    for (b, i, _k, _c, v) in [(b, i, 2, cid, float((7 * i + b) % 128)) for i in range(0, n, 3) for b in range(2, nb, 5)]:
        oscen[i].append((b, "param", S.P_DRAWBAR + 3, int(np.rint((127 - v) * 8.0 / 127.0))))
    sample = [0, 1, 3, 599, 1000, n - 1]
    tpl = Template(oracle, seed=7)
    oL, oR, *_ = oracle_run(oracle, tpl, [seeds[i] for i in sample], [sorted(oscen[i], key=lambda r: r[0]) for i in sample], nb)
    eL, xL = compare(outs[0][0][sample], oL)
    eR, xR = compare(outs[0][1][sample], oR)
    print(f"threaded dense events vs oracle ({len(sample)} instances): max|err| L={eL:.3g} R={eR:.3g}")
    assert max(eL, eR) <= TOL


def test_gpu_mixed_events_threaded_full_and_patched_entries(oracle):
    """The threaded front end sends a control delta as a 24-B record when only what a key
    or drawbar step changes has changed, and k_tgctl rebuilds its entry from the entry
    before it; any other change travels as a full entry.  1100 instances, 70 blocks: a key
    change on every block (records) mixed with overdrive character, rotor speed (a one-shot
    field), reverb mix, swell and percussion changes (full entries and routing patches) at
    staggered blocks.  Bit for bit against the serial front end (every delta a full entry)
    and against the oracle for a sample."""
    import os
    import torch
    import tunebfree_amd as T
    from orc_bind import Template
    n, nb = 1100, 70
    seeds = [5000 + i for i in range(n)]
    rows, oscen = [], [[] for _ in range(n)]

    def ev(b, i, kind, a, v):
        rows.append((b, i, 0 if kind == "note" else 1, a, float(v)))
        oscen[i].append((b, kind, a, v))

    for i in range(n):
        for (k, a, v) in S.jazz1_params():
            ev(0, i, k, a, v)
        for k in S.chord_for(i):
            ev(0, i, "note", k, 1)
        for b in range(1, nb):
            ev(b, i, "note", 60 + (i + b - 1) % 12, 0)
            ev(b, i, "note", 60 + (i + b) % 12, 1)
            if i % 3 == 0 and b % 6 == 0:
                ev(b, i, "param", S.P_CHARACTER, ((i + b) % 10) / 10.0)
            if i % 3 == 1 and b % 9 == 0:
                ev(b, i, "param", S.P_HORN, (b // 9) % 3)
            if i % 5 == 0 and b % 11 == 0:
                ev(b, i, "param", S.P_REVERB, ((i + b) % 7) / 7.0)
            if i % 7 == 0 and b % 10 == 0:
                ev(b, i, "param", S.P_SWELL, ((i + b) % 5) / 5.0)
            if i % 3 == 2 and b % 13 == 0:
                ev(b, i, "param", S.P_PERC, (b // 13) % 2)
    rows.sort(key=lambda r: r[0])
    outs = []
    for serial in (False, True):
        if serial:
            os.environ["TBF_HOST_SERIAL"] = "1"
        try:
            eng = T.Engine(sample_rate=48000.0, device=0)
        finally:
            os.environ.pop("TBF_HOST_SERIAL", None)
        tid = eng.template(seed=7)
        eng.add_instances([tid] * n, seeds)
        evs = eng.events(rows)
        L = torch.zeros((n, nb * 128), dtype=torch.float32, device="cuda")
        R = torch.zeros_like(L)
        eng.render_events_device(nb, evs, L.data_ptr(), R.data_ptr(), nb * 128)
        eng.synchronize()
        outs.append((L.cpu().numpy(), R.cpu().numpy()))
        eng.close()
        del L, R
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1].view(np.uint32), outs[1][1].view(np.uint32))
    sample = [0, 1, 2, 35, 700, n - 1]
    tpl = Template(oracle, seed=7)
    oL, oR, *_ = oracle_run(oracle, tpl, [seeds[i] for i in sample], [sorted(oscen[i], key=lambda r: r[0]) for i in sample], nb)
    eL, xL = compare(outs[0][0][sample], oL)
    eR, xR = compare(outs[0][1][sample], oR)
    print(f"mixed events, threaded vs oracle: max|err| L={eL:.3g} R={eR:.3g} bit-exact {xL:.6f} {xR:.6f}")
    assert max(eL, eR) <= TOL


def test_gpu_device_front_end_note_chunks(oracle):
    """Chunks whose events are all notes, over instances with no other control change
    pending, are stepped on the device (k_front): the messages, stepped blocks, control
    records and index table come from the key states at the chunk start and the events.
    1100 instances over 256 blocks (four chunks): the registration and first chords (host),
    a note-only chunk (device), a chunk with drawbar and percussion changes among the notes
    (host), a note-only chunk again (device); held keys re-pressed and releases of keys
    that are up included.  Bit for bit against the host
    front end (TBF_DEVICE_FRONT=0) and against the oracle for a sample."""
    import os
    import torch
    import tunebfree_amd as T
    from orc_bind import Template
    n, nb = 1100, 256
    seeds = [7000 + i for i in range(n)]
    rows, oscen = [], [[] for _ in range(n)]

    def ev(b, i, kind, a, v):
        rows.append((b, i, 0 if kind == "note" else 1, a, float(v)))
        oscen[i].append((b, kind, a, v))

    for i in range(n):
        for (k, a, v) in S.jazz1_params():
            ev(0, i, k, a, v)
        for k in S.chord_for(i):
            ev(0, i, "note", k, 1)
        for b in range(1, nb):
            if (i + b) % 3 == 0:
                continue  # a block without events: the block after one with messages still steps
            ev(b, i, "note", 55 + (i + b - 1) % 17, 0)
            ev(b, i, "note", 55 + (i + b) % 17, 1)
            if b % 5 == 0:
                ev(b, i, "note", 55 + (i + b) % 17, 1)  # a held key pressed again
            if b % 7 == 0:
                ev(b, i, "note", 100, 0)  # a key that is up
            if (i + b) % 11 == 0:  # keys outside [0, MAX_KEYS): ignored (src/tonegen.cpp:3098)
                bad = (-1, 384, 400, 4095)[(i + b) % 4]
                ev(b, i, "note", bad, 1)
                if b % 2:
                    ev(b, i, "note", bad, 0)
            if 128 <= b < 192 and b % 9 == 0 and i % 2 == 0:
                ev(b, i, "param", S.P_DRAWBAR + 2, (i + b) % 9)
            if 128 <= b < 192 and b % 16 == 0 and i % 3 == 0:
                ev(b, i, "param", S.P_PERC, (b // 16) % 2)
    rows.sort(key=lambda r: r[0])
    outs = []
    for front in (True, False):
        if not front:
            os.environ["TBF_DEVICE_FRONT"] = "0"
        try:
            eng = T.Engine(sample_rate=48000.0, device=0)
        finally:
            os.environ.pop("TBF_DEVICE_FRONT", None)
        tid = eng.template(seed=7)
        eng.add_instances([tid] * n, seeds)
        evs = eng.events(rows)
        L = torch.zeros((n, nb * 128), dtype=torch.float32, device="cuda")
        R = torch.zeros_like(L)
        eng.render_events_device(nb, evs, L.data_ptr(), R.data_ptr(), nb * 128)
        eng.synchronize()
        outs.append((L.cpu().numpy(), R.cpu().numpy()))
        eng.close()
        del L, R
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1].view(np.uint32), outs[1][1].view(np.uint32))
    sample = [0, 1, 2, 3, 550, n - 1]
    tpl = Template(oracle, seed=7)
    oL, oR, *_ = oracle_run(oracle, tpl, [seeds[i] for i in sample], [sorted(oscen[i], key=lambda r: r[0]) for i in sample], nb)
    eL, xL = compare(outs[0][0][sample], oL)
    eR, xR = compare(outs[0][1][sample], oR)
    print(f"device front end vs oracle: max|err| L={eL:.3g} R={eR:.3g} bit-exact {xL:.6f} {xR:.6f}")
    assert max(eL, eR) <= TOL


def test_gpu_device_front_end_param_events(oracle):
    """Chunks of notes, drawbar moves (upper and bus drawbars, the percussion trigger bus
    while percussion is on and off), vibrato switches and the percussion switches are
    stepped on the device (k_front, §8(f) row 1): 1100 instances over 192 blocks, a
    parameter event on most blocks of most instances.  Bit for bit against the host front
    end (TBF_DEVICE_FRONT=0) and against the oracle for a sample.  (Drawbar settings stay
    in 0..8: setDrawBar asserts that, src/tonegen.cpp:2741; the engine ignores others, and
    test_control_cpu covers that.)"""
    import os
    import torch
    import tunebfree_amd as T
    from orc_bind import Template
    n, nb = 1100, 192
    seeds = [9000 + i for i in range(n)]
    rows, oscen = [], [[] for _ in range(n)]

    def ev(b, i, kind, a, v):
        rows.append((b, i, 0 if kind == "note" else 1, a, float(v)))
        oscen[i].append((b, kind, a, v))

    for i in range(n):
        for (k, a, v) in S.jazz1_params():
            ev(0, i, k, a, v)
        for k in S.chord_for(i):
            ev(0, i, "note", k, 1)
        for b in range(1, nb):
            r = (i * 7 + b * 3) % 23
            if r < 9:
                ev(b, i, "param", S.P_DRAWBAR + r, (i + b) % 9)
            elif r < 12:
                ev(b, i, "param", S.P_BUS_DRAWBAR + 9 + (i + b) % 18, (i + 2 * b) % 9)  # lower / pedal buses
            elif r == 12:
                ev(b, i, "param", S.P_VIBRATO, (b // 12) % 2)
            elif r == 13:
                ev(b, i, "param", S.P_VIB_LOWER, (b // 17) % 2)
            elif r == 14:
                ev(b, i, "param", S.P_PERC, (b // 10) % 2)
            elif r == 15:
                ev(b, i, "param", S.P_PERC_HARM, (b // 13) % 2)
            elif r == 16:
                ev(b, i, "param", S.P_DRAWBAR + 8, (b % 9))  # the percussion trigger bus
            if b % 5 == 0:
                ev(b, i, "note", 55 + (i + b - 1) % 17, 0)
                ev(b, i, "note", 55 + (i + b) % 17, 1)
    rows.sort(key=lambda r: r[0])
    outs = []
    for front in (True, False):
        if not front:
            os.environ["TBF_DEVICE_FRONT"] = "0"
        try:
            eng = T.Engine(sample_rate=48000.0, device=0)
        finally:
            os.environ.pop("TBF_DEVICE_FRONT", None)
        tid = eng.template(seed=7)
        eng.add_instances([tid] * n, seeds)
        evs = eng.events(rows)
        L = torch.zeros((n, nb * 128), dtype=torch.float32, device="cuda")
        R = torch.zeros_like(L)
        eng.render_events_device(nb, evs, L.data_ptr(), R.data_ptr(), nb * 128)
        eng.synchronize()
        outs.append((L.cpu().numpy(), R.cpu().numpy()))
        eng.close()
        del L, R
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1].view(np.uint32), outs[1][1].view(np.uint32))
    sample = [0, 1, 2, 3, 550, n - 1]
    tpl = Template(oracle, seed=7)
    oL, oR, *_ = oracle_run(oracle, tpl, [seeds[i] for i in sample], [sorted(oscen[i], key=lambda r: r[0]) for i in sample], nb)
    eL, xL = compare(outs[0][0][sample], oL)
    eR, xR = compare(outs[0][1][sample], oR)
    print(f"device front end (params) vs oracle: max|err| L={eL:.3g} R={eR:.3g} bit-exact {xL:.6f} {xR:.6f}")
    assert max(eL, eR) <= TOL


def test_gpu_device_front_end_effect_events(oracle):
    """The effect setters on the device front end (k_front): rotary
    speed (drum / horn -> useRevOption, src/whirl.cpp:174-235), overdrive on / off and
    character (src/overdrive.cpp:387, 552-574), reverb mix (src/reverb.cpp:233), percussion
    volume and decay (src/tonegen.cpp:1725-1765), swell, whirl bypass and the vibrato type,
    mixed with notes and drawbars into >= 1024-event chunks over 1100 instances.  Every
    chunk after the first (fresh instances start dirty) is stepped on the device, except
    one with a character outside [0, 1] (the host front end, from the device chunks'
    mirror state).  Bit for bit against TBF_DEVICE_FRONT=0 and the oracle."""
    import os
    import torch
    import tunebfree_amd as T
    from orc_bind import Template
    n, nb = 1100, 256
    seeds = [9500 + i for i in range(n)]
    rows, oscen = [], [[] for _ in range(n)]

    def ev(b, i, kind, a, v):
        rows.append((b, i, 0 if kind == "note" else 1, a, float(v)))
        oscen[i].append((b, kind, a, v))

    for i in range(n):
        for (k, a, v) in S.jazz1_params():
            ev(0, i, k, a, v)
        for k in S.chord_for(i):
            ev(0, i, "note", k, 1)
        for b in range(1, nb):
            r = (i * 5 + b * 7) % 29
            if r == 0:
                ev(b, i, "param", S.P_DRUM, (b // 20 + i) % 3)
            elif r == 1:
                ev(b, i, "param", S.P_HORN, (b // 24 + i) % 3)
            elif r == 2:
                ev(b, i, "param", S.P_OVERDRIVE, (b // 30) % 2)
            elif r == 3:
                # character in [0, 1]; at block 200 instance 7 takes 1.5 (outside: the host front end)
                ev(b, i, "param", S.P_CHARACTER, ((i + b) % 11) / 10.0)
            elif r == 4:
                ev(b, i, "param", S.P_REVERB, ((i * 3 + b) % 9) / 8.0)
            elif r == 5:
                ev(b, i, "param", S.P_PERC_VOL, (b // 16) % 2)
            elif r == 6:
                ev(b, i, "param", S.P_PERC_DECAY, (b // 18) % 2)
            elif r == 7:
                ev(b, i, "param", S.P_SWELL, ((i + 2 * b) % 17) / 16.0)
            elif r == 8 and b % 64 == 8:
                ev(b, i, "param", S.P_WHIRL_BYPASS, (b // 64) % 2)
            elif r == 9:
                ev(b, i, "param", S.P_VIBRATO_TYPE, (i + b) % 7)  # 6: ignored by setVibrato
            elif r == 10:
                ev(b, i, "param", S.P_DRAWBAR + (i + b) % 9, (i + b) % 9)
            elif r == 11:
                ev(b, i, "param", S.P_PERC, (b // 22) % 2)
            if b % 6 == 0:
                ev(b, i, "note", 55 + (i + b - 1) % 17, 0)
                ev(b, i, "note", 55 + (i + b) % 17, 1)
    ev(200, 7, "param", S.P_CHARACTER, 1.5)
    rows.sort(key=lambda r: r[0])
    for o in oscen:
        o.sort(key=lambda r: r[0])
    outs, chunks = [], []
    for front in (True, False):
        if not front:
            os.environ["TBF_DEVICE_FRONT"] = "0"
        try:
            eng = T.Engine(sample_rate=48000.0, device=0)
        finally:
            os.environ.pop("TBF_DEVICE_FRONT", None)
        tid = eng.template(seed=7)
        eng.add_instances([tid] * n, seeds)
        evs = eng.events(rows)
        L = torch.zeros((n, nb * 128), dtype=torch.float32, device="cuda")
        R = torch.zeros_like(L)
        eng.render_events_device(nb, evs, L.data_ptr(), R.data_ptr(), nb * 128)
        eng.synchronize()
        outs.append((L.cpu().numpy(), R.cpu().numpy()))
        chunks.append(eng.front_chunks())
        eng.close()
        del L, R
    print(f"front-end chunks (device, host): device front on {chunks[0]}, off {chunks[1]}")
    assert chunks[0][0] >= 2 and chunks[0][1] >= 2, chunks  # the first chunk and block 200's: host
    assert chunks[1][0] == 0
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1].view(np.uint32), outs[1][1].view(np.uint32))
    sample = [0, 1, 2, 7, 550, n - 1]
    tpl = Template(oracle, seed=7)
    oL, oR, *_ = oracle_run(oracle, tpl, [seeds[i] for i in sample], [oscen[i] for i in sample], nb)
    eL, xL = compare(outs[0][0][sample], oL)
    eR, xR = compare(outs[0][1][sample], oR)
    print(f"device front end (effects) vs oracle: max|err| L={eL:.3g} R={eR:.3g} bit-exact {xL:.6f} {xR:.6f}")
    assert max(eL, eR) <= TOL


def test_gpu_device_front_end_small_chunks(oracle):
    """The device front end's event gate (TBF_FRONT_MIN, default 64 events per chunk): 96
    instances with a note change, a drawbar move and a reverb / rotary setter now and then,
    so chunks 1 and 2 carry ~420 events each.  Those step on the device (k_front), bit for
    bit like TBF_DEVICE_FRONT=0 and the oracle; a chunk under the gate steps on the host."""
    import os
    import torch
    import tunebfree_amd as T
    from orc_bind import Template
    n, nb = 96, 256
    seeds = [7700 + i for i in range(n)]
    rows, oscen = [], [[] for _ in range(n)]

    def ev(b, i, kind, a, v):
        rows.append((b, i, 0 if kind == "note" else 1, a, float(v)))
        oscen[i].append((b, kind, a, v))

    for i in range(n):
        for (k, a, v) in S.jazz1_params():
            ev(0, i, k, a, v)
        for k in S.chord_for(i):
            ev(0, i, "note", k, 1)
        for b in range(1, 192):
            if (b + i) % 40 == 0:
                ev(b, i, "note", 60 + (b // 40 + i) % 12, 0)
                ev(b, i, "note", 61 + (b // 40 + i) % 12, 1)
            if (b * 3 + i) % 97 == 0:
                ev(b, i, "param", S.P_DRAWBAR + (i + b) % 9, (i + b) % 9)
            if (b * 5 + i) % 131 == 0:
                ev(b, i, "param", S.P_REVERB if i % 2 else S.P_DRUM, (b % 3) / 2.0 if i % 2 else (b // 50) % 3)
    ev(250, 3, "note", 40, 1)  # the last chunk: a lone event, under the gate
    rows.sort(key=lambda r: r[0])
    for o in oscen:
        o.sort(key=lambda r: r[0])
    per_chunk = np.bincount([r[0] // 64 for r in rows], minlength=4)
    assert (per_chunk[1:3] >= 64).all() and per_chunk[3] < 64, per_chunk
    outs, chunks = [], []
    for front in (True, False):
        if not front:
            os.environ["TBF_DEVICE_FRONT"] = "0"
        try:
            eng = T.Engine(sample_rate=48000.0, device=0)
        finally:
            os.environ.pop("TBF_DEVICE_FRONT", None)
        tid = eng.template(seed=7)
        eng.add_instances([tid] * n, seeds)
        evs = eng.events(rows)
        L = torch.zeros((n, nb * 128), dtype=torch.float32, device="cuda")
        R = torch.zeros_like(L)
        eng.render_events_device(nb, evs, L.data_ptr(), R.data_ptr(), nb * 128)
        eng.synchronize()
        outs.append((L.cpu().numpy(), R.cpu().numpy()))
        chunks.append(eng.front_chunks())
        eng.close()
        del L, R
    print(f"front-end chunks (device, host): device front on {chunks[0]}, off {chunks[1]}")
    assert chunks[0][0] >= 2 and chunks[1][0] == 0, chunks
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1].view(np.uint32), outs[1][1].view(np.uint32))
    sample = [0, 3, 41, n - 1]
    tpl = Template(oracle, seed=7)
    oL, oR, *_ = oracle_run(oracle, tpl, [seeds[i] for i in sample], [oscen[i] for i in sample], nb)
    eL, xL = compare(outs[0][0][sample], oL)
    eR, xR = compare(outs[0][1][sample], oR)
    print(f"small device front-end chunks vs oracle: max|err| L={eL:.3g} R={eR:.3g} bit-exact {xL:.6f} {xR:.6f}")
    assert max(eL, eR) <= TOL


def test_gpu_steady_chunks(oracle):
    """A chunk in which no instance's control changes (every block plays each instance's
    current entry) runs up to TBF_STEADY_CHUNK blocks (default 512, at most 2048) per
    launch instead of 64, and ends at the next event's block.  Events at blocks 0..48
    (chords, drawbars, rotary, a note-off), then a reverb change and a whirl bypass toggle
    at blocks 300 / 330 / 340 inside one 450-block call, and a second call of 2100 blocks
    (four default 512-block chunks and a remainder; one 2048-block chunk at TBF_STEADY_CHUNK=2048):
    bit for bit the render of 64-block chunks (TBF_STEADY_CHUNK=64), and the oracle."""
    import os
    import torch
    import tunebfree_amd as T
    from orc_bind import Template
    n, nb1, nb2 = 48, 450, 2100
    seeds = [5000 + i for i in range(n)]
    oscen = [S.event_scenario(i) if i % 2 else S.bench_scenario(i) for i in range(n)]
    for i in (3, 10):
        oscen[i] = oscen[i] + [(300, "param", S.P_REVERB, 0.6)]
    for i in (5, 10):
        oscen[i] = oscen[i] + [(330, "param", S.P_WHIRL_BYPASS, 1), (340, "param", S.P_WHIRL_BYPASS, 0)]
    rows = sorted(((b, i, 0 if k == "note" else 1, a, float(v)) for i, sc in enumerate(oscen) for (b, k, a, v) in sc),
                  key=lambda r: r[0])
    outs = []
    for steady in (None, "2048", "64"):
        if steady:
            os.environ["TBF_STEADY_CHUNK"] = steady
        try:
            eng = T.Engine(sample_rate=48000.0, device=0)
        finally:
            os.environ.pop("TBF_STEADY_CHUNK", None)
        tid = eng.template(seed=7)
        eng.add_instances([tid] * n, seeds)
        evs = eng.events(rows)
        L = torch.zeros((n, (nb1 + nb2) * 128), dtype=torch.float32, device="cuda")
        R = torch.zeros_like(L)
        eng.render_events_device(nb1, evs, L.data_ptr(), R.data_ptr(), (nb1 + nb2) * 128)
        eng.render_device(nb2, L[:, nb1 * 128:].data_ptr(), R[:, nb1 * 128:].data_ptr(), (nb1 + nb2) * 128)
        eng.synchronize()
        outs.append((L.cpu().numpy(), R.cpu().numpy()))
        eng.close()
        del L, R
    for o in outs[:2]:
        assert np.array_equal(o[0].view(np.uint32), outs[2][0].view(np.uint32))
        assert np.array_equal(o[1].view(np.uint32), outs[2][1].view(np.uint32))
    sample = [0, 3, 5, 10, n - 1]
    tpl = Template(oracle, seed=7)
    oL, oR, *_ = oracle_run(oracle, tpl, [seeds[i] for i in sample], [sorted(oscen[i], key=lambda r: r[0]) for i in sample],
                            nb1 + nb2)
    eL, xL = compare(outs[0][0][sample], oL)
    eR, xR = compare(outs[0][1][sample], oR)
    print(f"steady chunks vs oracle: max|err| L={eL:.3g} R={eR:.3g} bit-exact {xL:.6f} {xR:.6f}")
    assert max(eL, eR) <= TOL


def test_gpu_set_steady_chunk_at_runtime(oracle):
    """tbf_set_steady_chunk between renders (bench.py toggles it): render, shrink to 64
    blocks (the stage buffers freed and reallocated at a smaller stride), render, grow to
    2048 and to 512 (reallocated larger, single and double sets re-derived), render: bit
    for bit the same calls on an engine fixed at TBF_STEADY_CHUNK=64, and the oracle.  The
    value returned is the one in effect (tbf_debug_chunks)."""
    import ctypes as C
    import os
    import torch
    import tunebfree_amd as T
    from orc_bind import Template
    lib = T.load_library()
    lib.tbf_debug_chunks.restype = C.c_int
    lib.tbf_debug_chunks.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    n, steps = 24, (300, 130, 700, 520)
    seeds = [7000 + i for i in range(n)]
    scens = [S.bench_scenario(i) for i in range(n)]
    total = sum(steps)
    outs = []
    for fixed in (False, True):
        if fixed:
            os.environ["TBF_STEADY_CHUNK"] = "64"
        try:
            eng = T.Engine(sample_rate=48000.0, device=0)
        finally:
            os.environ.pop("TBF_STEADY_CHUNK", None)
        tid = eng.template(seed=7)
        eng.add_instances([tid] * n, seeds)
        for i, sc in enumerate(scens):
            for (_, kind, a, v) in sc:
                (eng.note if kind == "note" else eng.set_param)(i, a, v)
        L = torch.zeros((n, total * 128), dtype=torch.float32, device="cuda")
        R = torch.zeros_like(L)
        off = 0
        for k, nb in enumerate(steps):
            if not fixed and k > 0:
                want = (64, 2048, 512)[k - 1]
                got = eng.set_steady_chunk(want)
                sb = C.c_uint32()
                assert lib.tbf_debug_chunks(eng._h, None, C.byref(sb)) == 0
                assert got == sb.value and got == want, (got, sb.value, want)
            eng.render_device(nb, L[:, off * 128:].data_ptr(), R[:, off * 128:].data_ptr(), total * 128)
            off += nb
        eng.synchronize()
        outs.append((L.cpu().numpy(), R.cpu().numpy()))
        eng.close()
        del L, R
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1].view(np.uint32), outs[1][1].view(np.uint32))
    pick = [0, 11, n - 1]
    oL, oR, *_ = oracle_run(oracle, Template(oracle, seed=7), [seeds[i] for i in pick], [scens[i] for i in pick], total)
    eL, xL = compare(outs[0][0][pick], oL)
    eR, xR = compare(outs[0][1][pick], oR)
    print(f"set_steady_chunk at runtime vs oracle: max|err| L={eL:.3g} R={eR:.3g} bit-exact {xL:.6f} {xR:.6f}")
    assert max(eL, eR) <= TOL


def test_gpu_threaded_host_control_reports_errors():
    """A bad event met by a host worker (threaded front end, >= 1024 instances) fails the
    call with the worker's message, as the serial loop would (the message is thread-local)."""
    import torch
    import tunebfree_amd as T
    n = 1100
    eng = T.Engine(sample_rate=48000.0, device=0)
    tid = eng.template(seed=7)
    eng.add_instances([tid] * n, [9000 + i for i in range(n)])
    rows = [(b, i, 0, 60 + (i + b) % 12, float(b % 2)) for i in range(n) for b in range(0, 8)]
    rows.append((3, 600, 1, 999, 1.0))  # no such parameter id
    L = torch.zeros((n, 8 * 128), dtype=torch.float32, device="cuda")
    R = torch.zeros_like(L)
    with pytest.raises(T.engine.TbfError, match="unknown parameter id"):
        eng.render_events_device(8, eng.events(rows), L.data_ptr(), R.data_ptr(), 8 * 128)
    eng.synchronize()
    eng.close()


def test_gpu_engine_switches_bitexact(oracle):
    """The scheduling switches change where and when work runs, never the output: with
    1100 instances, events on every block (keys, drawbars, control functions) and a
    programme change in the second chunk (that chunk's host control falls back to the
    serial loop), rendered in two calls, every switch renders bit-identically to the
    default engine: the serial host loop, the opt-in control stream (three persistent
    program slots), a third stage-buffer set, the chunk-parity streams, no pipelining,
    the streaming reverb network kernel (k_rv_core instead of k_rv_core_lds), the LDS
    kernel run alone or beside k_whirl only, and four stage-group streams.
    Instances without a programme change are also checked against the oracle."""
    import os
    import torch
    import tunebfree_amd as T
    from orc_bind import Template
    from test_control_cpu import PGM
    n, nb, split = 1100, 72, 40
    seeds = [5000 + i for i in range(n)]
    rows, oscen = [], [[] for _ in range(n)]
    for i in range(n):
        for (k, a, v) in S.jazz1_params():
            rows.append((0, i, 1, a, float(v)))
            oscen[i].append((0, k, a, v))
        for k in S.chord_for(i):
            rows.append((0, i, 0, k, 1.0))
            oscen[i].append((0, "note", k, 1))
        for b in range(1, nb):
            k0, k1 = 60 + (2 * i + b - 1) % 24, 60 + (2 * i + b) % 24
            rows.append((b, i, 0, k0, 0.0))
            oscen[i].append((b, "note", k0, 0))
            rows.append((b, i, 0, k1, 1.0))
            oscen[i].append((b, "note", k1, 1))
            if b % 4 == i % 4:
                rows.append((b, i, 1, S.P_DRAWBAR + 6, float((i + b) % 9)))
                oscen[i].append((b, "param", S.P_DRAWBAR + 6, (i + b) % 9))
    prog_inst = {5, 700}
    switches = [{}, {"TBF_HOST_SERIAL": "1"}, {"TBF_CTL_STREAM": "1"}, {"TBF_STAGE_BUFS": "3"},
                {"TBF_PIPE_MODE": "0"}, {"TBF_PIPELINE": "0"}, {"TBF_RV_LDS": "0"}, {"TBF_RV_EXCL": "1"},
                {"TBF_RV_EXCL": "2"}, {"TBF_PIPE_GROUPS": "0,1,2,3,3"}]
    outs, cid = [], None
    for env in switches:
        os.environ.update(env)
        try:
            eng = T.Engine(sample_rate=48000.0, device=0)
        finally:
            for k in env:
                os.environ.pop(k, None)
        assert eng.program_parse(PGM) == 4
        tid = eng.template(seed=7)
        eng.add_instances([tid] * n, seeds)
        cid = eng.control_id("upper.drawbar4")
        extra = [(b, i, 2, cid, float((3 * i + b) % 128)) for i in range(0, n, 5) for b in range(3, nb, 7)]
        extra += [(66, i, 3, 2, 0.0) for i in prog_inst]  # programme 2 in the second chunk
        ev = eng.events(rows + extra)
        L = torch.zeros((n, nb * 128), dtype=torch.float32, device="cuda")
        R = torch.zeros_like(L)
        first = ev[ev["block"] < split]
        rest = ev[ev["block"] >= split].copy()
        rest["block"] -= split
        eng.render_events_device(split, first, L.data_ptr(), R.data_ptr(), nb * 128)
        eng.render_events_device(nb - split, rest, L[:, split * 128:].data_ptr(), R[:, split * 128:].data_ptr(),
                                 nb * 128)
        eng.synchronize()
        outs.append((L.cpu().numpy(), R.cpu().numpy()))
        eng.close()
        del L, R
    for env, (l, r) in zip(switches[1:], outs[1:]):
        same = np.array_equal(l.view(np.uint32), outs[0][0].view(np.uint32)) and \
            np.array_equal(r.view(np.uint32), outs[0][1].view(np.uint32))
        print(f"{env}: bit-identical to the default engine: {same}")
        assert same, env
    for (b, i, _k, _c, v) in [(b, i, 2, cid, float((3 * i + b) % 128)) for i in range(0, n, 5) for b in range(3, nb, 7)]:
        oscen[i].append((b, "param", S.P_DRAWBAR + 3, int(np.rint((127 - v) * 8.0 / 127.0))))
    sample = [0, 1, 4, 550, 1099]
    tpl = Template(oracle, seed=7)
    oL, oR, *_ = oracle_run(oracle, tpl, [seeds[i] for i in sample], [sorted(oscen[i], key=lambda r: r[0]) for i in sample], nb)
    eL, _ = compare(outs[0][0][sample], oL)
    eR, _ = compare(outs[0][1][sample], oR)
    print(f"switches scenario vs oracle ({len(sample)} instances): max|err| L={eL:.3g} R={eR:.3g}")
    assert max(eL, eR) <= TOL


def test_gpu_synth_sound_irregular_periods(oracle, tunings):
    """tbf_synth_sound (the synthSound FIFO of b_synth/lv2.cpp:1270-1287) with irregular
    period sizes (1 .. 700 frames; a call that needs several blocks renders them in one
    launch), events and an MTS-ESP retune between calls: each lands at the next block the
    FIFO renders, so the stream equals the oracle's block-by-block render with the events
    at those blocks."""
    from orc_bind import Template
    m19 = np.asarray(tunings["19TET"], np.float64)
    n = 3
    eng = _engine()
    tid = eng.template(seed=7)
    tid19 = eng.template(mts128=m19, seed=8)
    seeds = [2000 + i for i in range(n)]
    eng.add_instances([tid] * n, seeds)
    t12, t19 = Template(oracle, seed=7), Template(oracle, mts128=m19, seed=8)
    rng = np.random.default_rng(5)
    periods = [int(x) for x in rng.choice([1, 37, 64, 128, 129, 256, 300, 515, 700], size=40)]
    consumed, outL, outR = 0, [], []
    oscen = [[] for _ in range(n)]
    for c, nf in enumerate(periods):
        blk = -(-consumed // 128)  # the next block the FIFO renders
        evs = []
        if c == 0:
            evs += [(k, a, v) for (k, a, v) in S.jazz1_params()]
        if c % 4 == 0:
            evs += [("note", k, 1) for k in S.chord_for(c)]
        if c % 4 == 2:
            evs += [("note", k, 0) for k in S.chord_for(c - 2)]
        if c % 7 == 3:
            evs += [("param", S.P_DRAWBAR + 2, c % 9)]
        if c == 20:
            evs += [("retune", 1, 0)]
        for i in range(n):
            for (k, a, v) in evs:
                if k == "note":
                    eng.note(i, a + i, v)
                    oscen[i].append((blk, k, a + i, v))
                elif k == "retune":
                    eng.retune(i, tid19)
                    oscen[i].append((blk, k, a, v))
                else:
                    eng.set_param(i, a, v)
                    oscen[i].append((blk, k, a, v))
        L, R = eng.synth_sound(nf)
        outL.append(L)
        outR.append(R)
        consumed += nf
    L, R = np.concatenate(outL, axis=1), np.concatenate(outR, axis=1)
    nb = -(-consumed // 128)
    oL, oR, *_ = oracle_run(oracle, t12, seeds, oscen, nb, templates=[t12, t19])
    eL, xL = compare(L, oL[:, :consumed])
    eR, xR = compare(R, oR[:, :consumed])
    print(f"synth_sound {len(periods)} periods / {consumed} frames: max|err| L={eL:.3g} R={eR:.3g} "
          f"bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL
    eng.close()


def test_gpu_lv2_synth_sound_run_loop(oracle):
    """The LV2 binding of INTEGRATION.md section 2, compiled verbatim (libtbf_lv2.so),
    driven like the plugin's run() (b_synth/lv2.cpp:1120-1140): per period, for each MIDI
    event at frame t, `written = synthSound (b3s, written, t)` when written + 128 < t < n,
    then the event; finally `written = synthSound (b3s, written, n)`.  Irregular periods
    (1 .. 700 frames) and events inside them: each event lands at the next block the FIFO
    renders, so the audio equals the oracle's render with the events at those blocks."""
    import ctypes as C
    from pathlib import Path
    import tunebfree_amd as T
    from orc_bind import Template
    lv2 = C.CDLL(str(Path(__file__).resolve().parents[1] / "tunebfree_amd" / "libtbf_lv2.so"))
    lv2.tbf_lv2_synth_sound.restype = C.c_uint32
    lv2.tbf_lv2_synth_sound.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p]
    lv2.tbf_lv2_key.restype = None
    lv2.tbf_lv2_key.argtypes = [C.c_void_p, C.c_int, C.c_int]
    lv2.tbf_lv2_instantiate.restype = C.c_void_p
    lv2.tbf_lv2_instantiate.argtypes = [C.c_double]
    # tbf_instantiate_engine itself (seeded by time(NULL), so no oracle twin): it must build
    # and render finite audio through synthSound
    h = lv2.tbf_lv2_instantiate(48000.0)
    assert h
    buf = np.zeros((2, 300), np.float32)
    lv2.tbf_lv2_key(h, 60, 1)
    assert lv2.tbf_lv2_synth_sound(h, 0, 300, buf[0].ctypes.data, buf[1].ctypes.data) == 300
    assert np.isfinite(buf).all()
    T.load_library().tbf_engine_destroy(C.c_void_p(h))

    eng = _engine()
    tid = eng.template(seed=7)
    eng.add_instances([tid], [3001])
    tpl = Template(oracle, seed=7)
    for (k, a, v) in S.jazz1_params():
        eng.set_param(0, a, v)
    oscen = [[(0, k, a, v) for (k, a, v) in S.jazz1_params()]]
    rng = np.random.default_rng(11)
    served, out = 0, []  # frames the FIFO has served
    keys_down = []
    for c in range(48):
        n = int(rng.choice([1, 37, 64, 128, 129, 256, 300, 515, 700]))
        L = np.zeros(n, np.float32)
        R = np.zeros(n, np.float32)
        nev = int(rng.integers(0, 3))
        frames = sorted(int(x) for x in rng.integers(0, n, size=nev))
        written = 0
        for t in frames:
            if written + 128 < t < n:
                written = lv2.tbf_lv2_synth_sound(eng._h, written, t, L.ctypes.data, R.ctypes.data)
            key = 48 + int(rng.integers(0, 36))
            on = 0 if (keys_down and rng.random() < 0.4) else 1
            if not on:
                key = keys_down.pop(0)
            else:
                keys_down.append(key)
            lv2.tbf_lv2_key(eng._h, key, on)
            oscen[0].append((-(-(served + written) // 128), "note", key, on))
        written = lv2.tbf_lv2_synth_sound(eng._h, written, n, L.ctypes.data, R.ctypes.data)
        assert written == n
        served += n
        out.append((L, R))
    L = np.concatenate([o[0] for o in out])[None]
    R = np.concatenate([o[1] for o in out])[None]
    nb = -(-served // 128)
    oL, oR, *_ = oracle_run(oracle, tpl, [3001], oscen, nb)
    eL, xL = compare(L, oL[:, :served])
    eR, xR = compare(R, oR[:, :served])
    print(f"lv2 run loop: {served} frames, {len(oscen[0])} events: max|err| L={eL:.3g} R={eR:.3g} "
          f"bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL
    eng.close()


def test_gpu_cli_host_synth_sound(oracle, tmp_path):
    """§8(f) row 3: the headless host shell (tunebfree_amd/tbf_cli, the counterpart of
    src/main.cpp:243-292 and b_synth/lv2.cpp:212-239) pulls 256-frame periods through
    tbf_synth_sound after installing a programme; its audio equals the oracle's."""
    import subprocess
    from pathlib import Path
    from orc_bind import Chain, Template
    from test_control_cpu import PGM
    cli = Path(__file__).resolve().parents[1] / "tunebfree_amd" / "tbf_cli"
    assert cli.exists(), "tbf_cli not built"
    (tmp_path / "t.pgm").write_text(PGM)
    nb, buf, n = 24, 256, 2
    frames = nb * 128
    subprocess.run([str(cli), "--pgm", str(tmp_path / "t.pgm"), "--program", "0", "--instances", str(n),
                    "--buffer", str(buf), "--seconds", str(frames / 48000.0), "--seed", "5",
                    "--character", "0.5", "--raw", str(tmp_path / "o.raw")], check=True, timeout=120)
    raw = np.fromfile(tmp_path / "o.raw", np.float32)
    L = np.zeros((n, frames), np.float32)
    R = np.zeros((n, frames), np.float32)
    pos, done = 0, 0
    while done < frames:
        nf = min(buf, frames - done)
        blk = raw[pos: pos + n * nf * 2].reshape(n, nf, 2)
        L[:, done:done + nf], R[:, done:done + nf] = blk[..., 0], blk[..., 1]
        pos += n * nf * 2
        done += nf
    tpl = Template(oracle, seed=5)
    worst = 0.0
    for i in range(n):
        ch = Chain(oracle, tpl, 5 + 1000 + i)
        for (kind, a, v) in S.jazz1_params():
            ch.param(a, v)
        for k in (60, 64, 67, 72):
            ch.note(k, 1)
        oL, oR = ch.render(nb)
        worst = max(worst, compare(L[i], oL)[0], compare(R[i], oR)[0])
    print(f"cli host: max|err|={worst:.3g}")
    assert worst <= TOL


def _random_mts(seed):
    """A seeded random MTS-ESP table: 12-TET moved by a random transposition (-700 ..
    +700 cents) and per-key offsets (-50 .. +50 cents), so the wheels' sine arguments
    cover ranges the fixed tunings do not."""
    r = np.random.default_rng(seed)
    cents = r.uniform(-700, 700) + r.uniform(-50, 50, 128)
    return 440.0 * 2.0 ** ((np.arange(128) - 69) / 12.0 + cents / 1200.0)


def _oracle_bank_worker(args):
    sr, seeds = args
    import hashlib
    from orc_bind import Template, load_oracle
    lib = load_oracle()
    out = []
    for sd in seeds:
        b, l = Template(lib, sr=sr, mts128=_random_mts(sd), seed=sd).bank()
        out.append((sd, b.astype(np.float32).tobytes(), np.asarray(l).tobytes()))
    return out


@pytest.mark.parametrize("sr", [48000.0, 96000.0])
def test_gpu_device_banks_random_mts_no_flips(oracle, sr):
    """the device wave banks (k_tpl_wave: FP64 sin of the device library,
    rounded to float) against the oracle's (glibc sin) for 200 seeded random MTS tables
    per sample rate: the number of float samples that differ (a 1-ulp FP64 sin
    difference flipping a float rounding) must be 0."""
    import multiprocessing as mp
    import os
    import tunebfree_amd as T
    seeds = [7000 + int(sr) // 1000 * 1000 + k for k in range(200)]
    workers = max(1, min(16, (os.cpu_count() or 1)))
    parts = [seeds[k::workers] for k in range(workers)]
    with mp.get_context("spawn").Pool(workers) as pool:
        ref = {sd: (b, l) for part in pool.map(_oracle_bank_worker, [(sr, p) for p in parts]) for sd, b, l in part}
    eng = T.Engine(sample_rate=sr, device=0)
    ids = eng.templates(seeds, mts128=np.stack([_random_mts(sd) for sd in seeds]))
    flips, samples, worst = 0, 0, 0.0
    for tid, sd in zip(ids, seeds):
        bank, lens = eng.template_bank(tid)
        ob = np.frombuffer(ref[sd][0], np.float32)
        ol = np.frombuffer(ref[sd][1], np.asarray(lens).dtype)
        assert np.array_equal(np.asarray(lens), ol), sd
        assert bank.shape == ob.shape, sd
        d = bank.view(np.uint32) != ob.view(np.uint32)
        flips += int(d.sum())
        samples += bank.size
        if d.any():
            worst = max(worst, float(np.abs(bank[d].astype(np.float64) - ob[d]).max()))
    eng.close()
    print(f"device banks, {len(seeds)} random MTS tables at {sr:.0f} Hz: {samples} samples, "
          f"{flips} differ from the oracle (max |diff| {worst:.3g})")
    assert flips == 0


@pytest.mark.parametrize("sr", [48000.0, 96000.0])
def test_gpu_device_templates_match_oracle_and_reference(oracle, sr):
    """§8(f) row 2: templates built on the device (tbf_templates_create: per-chunk
    jumps of the glibc rand() stream + the writeSamples sines) against
      - the oracle's template builder, bit for bit (wave bank, wheel lengths,
        envelopes, key-compression table), on the same (tuning, seed) inputs, and
      - the reference's own src/tonegen.cpp builders (digests committed in
        tests/golden/template_pins.json, generated by oracle/ref_tpl_pin.cpp): the 7
        tunings at this sample rate with their pinned seeds.
    A second batch (the 6 table tunings again with other seeds, plus three 12-TET
    templates) is checked against the oracle."""
    import ctypes as C
    import hashlib
    import json
    import time
    from pathlib import Path
    import tunebfree_amd as T
    from orc_bind import Template
    gold = Path(__file__).resolve().parent / "golden"
    tunings = json.loads((gold / "tunings.json").read_text())
    allpins = json.loads((gold / "template_pins.json").read_text())
    pins = [p for p in allpins if p["sr"] == sr and not p.get("cfg")]
    eng = T.Engine(sample_rate=sr, device=0)
    lib = T.load_library()
    lib.tbf_debug_tables.restype = C.c_int
    lib.tbf_debug_tables.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]

    from orc_bind import Cfg, contrib_from
    lib.tbf_debug_contrib.restype = C.c_int
    lib.tbf_debug_contrib.argtypes = [C.c_void_p, C.c_uint32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_uint32]

    def tables(tid):
        bank, lens = eng.template_bank(tid)
        a, r, k = np.zeros((9, 128), np.float32), np.zeros((9, 128), np.float32), np.zeros(128, np.float32)
        assert lib.tbf_debug_tables(eng._h, tid, a.ctypes.data, r.ctypes.data, k.ctypes.data) >= 0
        contrib = contrib_from(lambda kk, w, b, lv, cap: lib.tbf_debug_contrib(eng._h, tid, kk, w, b, lv, cap))
        return {"bank": bank, "lens": lens, "attack": a, "release": r, "keycomp": k, "contrib": contrib}

    def mts(nm):
        return None if tunings[nm] is None else np.asarray(tunings[nm], np.float64)

    # batch 1: the pinned (tuning, seed) cases; the 12-TET one has no MTS table, so it is
    # built in its own call (tbf_templates_create takes all-or-none frequency tables)
    table_pins = [p for p in pins if tunings[p["tuning"]] is not None]
    t0 = time.perf_counter()
    ids = eng.templates([p["seed"] for p in table_pins], mts128=np.stack([mts(p["tuning"]) for p in table_pins]))
    t_dev = time.perf_counter() - t0
    tet = [p for p in pins if tunings[p["tuning"]] is None]
    ids += eng.templates([p["seed"] for p in tet])
    cases = [(tid, p["tuning"], p["seed"], p) for tid, p in zip(ids, table_pins + tet)]
    # batch 2: other seeds, checked against the oracle only
    names = [k for k in sorted(tunings) if tunings[k] is not None]
    ids2 = eng.templates([500 + j for j in range(len(names))], mts128=np.stack([mts(nm) for nm in names]))
    ids2 += eng.templates([1, 2, 3])
    cases += [(tid, nm, 500 + j, None) for j, (tid, nm) in enumerate(zip(ids2, names))]
    cases += [(tid, "12TET", s, None) for tid, s in zip(ids2[len(names):], (1, 2, 3))]
    for tid, nm, seed, pin in cases:
        got = tables(tid)
        o = Template(oracle, sr=sr, mts128=mts(nm), seed=seed)
        ob, ol = o.bank()
        oa, orr, ok = o.envs()
        want = {"bank": ob, "lens": ol, "attack": oa, "release": orr, "keycomp": ok, "contrib": o.contrib()}
        for key in want:
            assert np.array_equal(np.asarray(got[key]).view(np.uint32), np.asarray(want[key]).view(np.uint32)), \
                (nm, seed, key)
            if pin is not None:
                assert hashlib.sha256(np.ascontiguousarray(got[key]).tobytes()).hexdigest() == pin[key], (nm, key)
    print(f"device templates @{sr:.0f}: {len(cases)} vs oracle, {len(pins)} vs reference pins; "
          f"first batch of {len(table_pins)} in {t_dev * 1e3:.1f} ms")
    eng.close()
    # the template cfg keys (envelope models, lengths, levels, x-precision; wheel EQ,
    # harmonics, the play matrix lists and levels) on the device path
    for p in [p for p in allpins if p["sr"] == sr and p.get("cfg")]:
        eng = T.Engine(sample_rate=sr, device=0)
        eng.config(S.CFG_SETS[p["cfg"]])
        m = mts(p["tuning"])
        tid = eng.templates([p["seed"]], mts128=None if m is None else m[None])[0]
        bank, lens = eng.template_bank(tid)
        a, r, k = np.zeros((9, 128), np.float32), np.zeros((9, 128), np.float32), np.zeros(128, np.float32)
        assert lib.tbf_debug_tables(eng._h, tid, a.ctypes.data, r.ctypes.data, k.ctypes.data) >= 0
        got = {"bank": bank, "lens": lens, "attack": a, "release": r, "keycomp": k}
        got["contrib"] = contrib_from(lambda kk, w, b, lv, cap: lib.tbf_debug_contrib(eng._h, tid, kk, w, b, lv, cap))
        o = Template(oracle, sr=sr, mts128=m, seed=p["seed"], cfg=Cfg(oracle, S.CFG_SETS[p["cfg"]]))
        ob, ol = o.bank()
        oa, orr, ok = o.envs()
        want = {"bank": ob, "lens": ol, "attack": oa, "release": orr, "keycomp": ok, "contrib": o.contrib()}
        for key, v in got.items():
            assert np.array_equal(np.asarray(v).view(np.uint32), np.asarray(want[key]).view(np.uint32)), (p["cfg"], key)
            assert hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest() == p[key], (p["cfg"], key)
        eng.close()


def test_gpu_device_play_matrix_matches_host_builder():
    """the play matrix built on the device (k_tpl_matrix in
    tbf_templates_create: applyManualDefaults' nearest-wheel search, the pedal defaults,
    the default crosstalk and compilePlayMatrix's cell sums, src/tonegen.cpp:707-879,
    1061-1213) against the host builder (tbf_template_create, pinned to the reference's
    compilePlayMatrix by tests/golden/template_pins.json), bit for bit over every key's
    (wheel, bus, level) list: detuned tunings and bus ratios away from the defaults, with
    the default cfg, the list keys (osc_lists) and the crosstalk / floor / minimum levels
    (osc_models).  Also times a 64-template batch against TBF_HOST_MATRIX=1."""
    import ctypes as C
    import os
    import time
    import tunebfree_amd as T
    from orc_bind import contrib_from
    lib = T.load_library()
    lib.tbf_debug_contrib.restype = C.c_int
    lib.tbf_debug_contrib.argtypes = [C.c_void_p, C.c_uint32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_uint32]
    rng = np.random.default_rng(8)
    tet = 440.0 * 2.0 ** ((np.arange(128) - 69) / 12.0)
    base = np.array([0.5, 1.5, 1, 2, 3, 4, 5, 6, 8])
    n = 8
    M = tet[None] * 2.0 ** (rng.uniform(-40, 40, (n, 128)) / 1200.0)
    M[1] = np.sort(tet * 2.0 ** (rng.uniform(-200, 200, 128) / 1200.0))  # far off the wheels
    R = base[None] * 2.0 ** (rng.uniform(-60, 60, (n, 9)) / 1200.0)
    R[2] = base                                                            # exact ratios
    R[3, 4] = R[3, 3]                                                      # two buses alike
    seeds = [900 + i for i in range(n)]
    for cfgname in (None, "osc_lists", "osc_models"):
        eng = T.Engine(sample_rate=48000.0, device=0)
        if cfgname:
            eng.config(S.CFG_SETS[cfgname])
        dev = eng.templates(seeds, mts128=M, ratio9=R)
        host = [eng.template(mts128=M[i], ratio9=R[i], seed=seeds[i]) for i in range(n)]
        for i in range(n):
            got, want = (contrib_from(lambda kk, w, b, lv, cap, t=t: lib.tbf_debug_contrib(eng._h, t, kk, w, b, lv, cap))
                         for t in (dev[i], host[i]))
            assert got.tobytes() == want.tobytes(), (cfgname, i)
        eng.close()
    eng = T.Engine(sample_rate=48000.0, device=0)
    eng.templates([1])  # warm: first launch, allocations
    ms = {}
    for mode in ("device", "host"):
        if mode == "host":
            os.environ["TBF_HOST_MATRIX"] = "1"
        try:
            t0 = time.perf_counter()
            eng.templates([2000 + i for i in range(64)])
            ms[mode] = (time.perf_counter() - t0) * 1e3
        finally:
            os.environ.pop("TBF_HOST_MATRIX", None)
    eng.close()
    print(f"64 templates (bank + play matrix): {ms['device']:.1f} ms with the device play matrix, "
          f"{ms['host']:.1f} ms with the host one")


def test_gpu_pipelined_chunks_across_calls(oracle):
    """Cross-chunk pipelining (stage k of a chunk on its own stream, overlapping later
    stages of earlier chunks and of the previous render call): back-to-back
    tbf_render_device calls of 70 blocks (a 64-block chunk plus a 6-block chunk, so
    both buffer parities alternate irregularly) on a torch stream with no host sync,
    then a synchronous render; bit-identical to the oracle."""
    import torch
    eng, tpl, seeds, scens = _setup(oracle, 6, S.bench_scenario)
    L0, R0 = engine_run(eng, scens, 1)  # block 0 carries the control uploads
    nb, calls = 70, 4
    L = torch.zeros((6, nb * calls * 128), dtype=torch.float32, device="cuda")
    R = torch.zeros_like(L)
    st = torch.cuda.Stream()
    stride = nb * calls * 128
    for c in range(calls):
        eng.render_device(nb, L[:, c * nb * 128:].data_ptr(), R[:, c * nb * 128:].data_ptr(), stride, st.cuda_stream)
    st.synchronize()
    L2, R2 = eng.render(3)
    gL = np.concatenate([L0, L.cpu().numpy(), L2], axis=1)
    gR = np.concatenate([R0, R.cpu().numpy(), R2], axis=1)
    total = 1 + nb * calls + 3
    oL, oR, *_ = oracle_run(oracle, tpl, seeds, scens, total)
    eL, xL = compare(gL, oL)
    eR, xR = compare(gR, oR)
    print(f"pipelined: {total} blocks, max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL


def test_gpu_reverb_network_group_boundaries(oracle):
    """k_rv_core_lds runs a launch in groups of eleven 64-sample sub-blocks, and launches
    of fewer than 8 blocks use k_rv_core; both keep the same ring and counter state.
    Render calls of 7, 8, 11, 12, 17, 22 and 33 blocks (14 sub-blocks on k_rv_core, then
    16 = 11 + 5, 22 = 2 x 11, 24 = 22 + 2, 34 = 33 + 1, 44 = 4 x 11, 66 = 6 x 11) switch
    kernels and end groups at every offset pattern: bit-identical to the oracle, and to an
    engine that runs k_rv_core throughout (TBF_RV_LDS=0)."""
    import os
    calls = [7, 8, 11, 12, 17, 22, 33]
    outs = []
    for env in ({}, {"TBF_RV_LDS": "0"}):
        os.environ.update(env)
        try:
            eng, tpl, seeds, scens = _setup(oracle, 6, S.bench_scenario)
        finally:
            for k in env:
                os.environ.pop(k, None)
        parts = [engine_run(eng, scens, 1)]  # block 0 carries the scenario's events
        parts += [eng.render(nb) for nb in calls]
        eng.close()
        outs.append((np.concatenate([p[0] for p in parts], axis=1), np.concatenate([p[1] for p in parts], axis=1)))
    total = 1 + sum(calls)
    oL, oR, *_ = oracle_run(oracle, tpl, seeds, scens, total)
    eL, xL = compare(outs[0][0], oL)
    eR, xR = compare(outs[0][1], oR)
    print(f"group boundaries: {total} blocks, max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_gpu_reverb_phase_binade_crossing(oracle):
    """A reverb vibrato phase that crosses a binade inside a launch (phases placed just
    below powers of two, both signs) makes k_rv_core_lds walk that group sub-block by
    sub-block; a sub-block after the crossing is closed-form with its new step and rows
    computed inline, exactly as k_rv_core does it.  So the LDS network kernel (one 64-block
    call, or 23 + 41), the streaming kernel (TBF_RV_LDS=0) and a 7 + 57 split (k_rv_core
    for the first call) are bit-identical, and all match the oracle (literal sin)."""
    import ctypes as C
    import os
    from orc_bind import Chain
    n, nb = 4, 64
    pokes = [(0, 0, 2.0 ** 20 - 0.5), (0, 3, -(2.0 ** 19) - 0.3), (1, 5, 2.0 ** 21 - 0.9), (1, 7, 2.0 ** 10 - 0.2)]
    runs = []
    for env, split in (({}, [64]), ({}, [23, 41]), ({}, [7, 57]), ({"TBF_RV_LDS": "0"}, [64])):
        os.environ.update(env)
        try:
            eng, tpl, seeds, scens = _setup(oracle, n, S.bench_scenario)
        finally:
            for k in env:
                os.environ.pop(k, None)
        for i in range(n):
            for (c, l, v) in pokes:
                eng.debug_reverb_phase(i, c, l, v - 0.0131 * i)
        parts = [engine_run(eng, scens, split[0])] + [eng.render(k) for k in split[1:]]
        assert eng.error_flags() & 8, "no phase run left its closed form: the crossing was not exercised"
        eng.close()
        runs.append((np.concatenate([p[0] for p in parts], axis=1), np.concatenate([p[1] for p in parts], axis=1)))
    fn = oracle.orc_debug_rv_phase
    fn.restype, fn.argtypes = None, [C.c_void_p, C.c_int, C.c_int, C.c_double]
    oL, oR = [], []
    for i, (seed, sc) in enumerate(zip(seeds, scens)):
        ch = Chain(oracle, tpl, seed)
        for (c, l, v) in pokes:
            fn(ch.ptr, c, l, v - 0.0131 * i)
        L, R, *_ = S.run(ch, sc, nb, stages=True)
        oL.append(L)
        oR.append(R)
    eL, xL = compare(runs[0][0], np.stack(oL))
    eR, xR = compare(runs[0][1], np.stack(oR))
    print(f"binade crossing: max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL
    for k, r in enumerate(runs[1:], 1):
        same = all(np.array_equal(a.view(np.uint32), b.view(np.uint32)) for a, b in zip(runs[0], r))
        print(f"variant {k}: bit-identical to the single LDS call: {same}")
        assert same


def test_gpu_full_size_bench_batch(oracle):
    """BASELINE configs[2] at its full size (4096 instances x 64 blocks, one call, the
    bench's render): instances spread over the whole batch (both ends and the middle of
    every stage buffer) match the oracle, and size-independent properties hold —
    instances are independent (an engine holding only the upper half renders those rows
    identically) and the result does not depend on how the blocks are split into
    calls (16 + 48 blocks, pipelined across the call boundary)."""
    n, nb = 4096, 64
    eng, tpl, seeds, scens = _setup(oracle, n, S.bench_scenario)
    L, R = engine_run(eng, scens, nb)
    assert L.shape == (n, nb * 128) and np.all(np.isfinite(L)) and np.all(np.isfinite(R))
    pick = [0, 1, 1023, 1365, 2047, 2048, 2730, 4094, 4095]
    oL, oR, *_ = oracle_run(oracle, tpl, [seeds[i] for i in pick], [scens[i] for i in pick], nb)
    eL, xL = compare(L[pick], oL)
    eR, xR = compare(R[pick], oR)
    print(f"full size: max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL

    half = n // 2
    import tunebfree_amd as T
    eng2 = T.Engine(sample_rate=48000.0, device=0, chain=0)
    tid = eng2.template(seed=7)
    eng2.add_instances([tid] * half, seeds[half:])
    for i, sc in enumerate(scens[half:]):
        for (b, kind, a, v) in sc:
            assert b == 0
            if kind == "note":
                eng2.note(i, a, v)
            else:
                eng2.set_param(i, a, v)
    L2a, R2a = eng2.render(16)
    L2b, R2b = eng2.render(nb - 16)
    L2 = np.concatenate([L2a, L2b], axis=1)
    R2 = np.concatenate([R2a, R2b], axis=1)
    assert np.array_equal(L2.view(np.uint32), L[half:].view(np.uint32))
    assert np.array_equal(R2.view(np.uint32), R[half:].view(np.uint32))
    eng2.close()

    # two more steady 64-block calls, as the bench's timed steps render them (no control
    # deltas: k_tonegen splits each instance's blocks over waves, all six stages pipelined
    # across chunks and calls, the network kernel persistent): still the oracle's samples
    more = [eng.render(nb) for _ in range(2)]
    pick = [0, 3, 2047, 4095]
    oL, oR, *_ = oracle_run(oracle, tpl, [seeds[i] for i in pick], [scens[i] for i in pick], 3 * nb)
    gL = np.concatenate([m[0][pick] for m in more], axis=1)
    gR = np.concatenate([m[1][pick] for m in more], axis=1)
    eL, xL = compare(gL, oL[:, nb * 128:])
    eR, xR = compare(gR, oR[:, nb * 128:])
    print(f"steady calls: max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL


@pytest.mark.parametrize("debug_flags", [0, 1])
def test_gpu_parameter_sweep(oracle, debug_flags):
    """Parameter regions the bench registration does not reach (scenarios.sweep_scenario):
    overdrive character 0 / 0.3 / 0.9 / 1.0 and clean, reverb mix 0 / 0.7 / 1.0,
    percussion normal/soft x fast/slow x 2nd/3rd with retriggers, 13-key clusters,
    pedal keys 256..383 with pedal drawbars, rotary stop <-> fast transitions; 12
    instances in one engine against the oracle, with the fast paths and with every
    guarded stage forced onto its serial replay (TBF_DEBUG_FORCE_SERIAL)."""
    import tunebfree_amd as T
    n, nb = 12, 72
    eng, tpl, seeds, scens = _setup(oracle, n, S.sweep_scenario, debug_flags=debug_flags)
    L, R = engine_run(eng, scens, nb)
    oL, oR, oA, oB, oC = oracle_run(oracle, tpl, seeds, scens, nb)
    eL, xL = compare(L, oL)
    eR, xR = compare(R, oR)
    flags = eng.error_flags()
    print(f"sweep (debug {debug_flags}): max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f} "
          f"paths 0x{flags:x}")
    assert max(eL, eR) <= TOL
    for i in range(n):  # every instance sounds (no silent pass through a broken stage)
        assert float(np.abs(oL[i]).max()) > 1e-3
    if debug_flags:
        want = T.engine.PATH_VIB_SERIAL | T.engine.PATH_WH_ANGLE | T.engine.PATH_WH_MOTION | T.engine.PATH_RV_PHASE
        assert flags & want == want, hex(flags)


def test_gpu_random_character_and_reverb_mix(oracle):
    """seeded random overdrive character (0..1) and reverb mix (0..1)
    per instance, changed mid-render, against the oracle: the overdrive's FP64 sin
    passes and the reverb's sin / asin on the device library across continuous parameter
    values, not only the fixed sweep points."""
    rng = np.random.default_rng(2024)
    n, nb = 16, 48
    ch = rng.uniform(0.0, 1.0, size=(n, 2))
    rv = rng.uniform(0.0, 1.0, size=(n, 2))

    def scen(i):
        ev = [(0, k, a, b) for (k, a, b) in S.jazz1_params(character=float(ch[i, 0]), reverb=float(rv[i, 0]))]
        ev += [(0, "note", k, 1) for k in S.chord_for(i)]
        ev += [(24, "param", S.P_CHARACTER, float(ch[i, 1])), (24, "param", S.P_REVERB, float(rv[i, 1]))]
        return ev
    eng, tpl, seeds, scens = _setup(oracle, n, scen)
    L, R = engine_run(eng, scens, nb)
    oL, oR, *_ = oracle_run(oracle, tpl, seeds, scens, nb)
    eL, xL = compare(L, oL)
    eR, xR = compare(R, oR)
    print(f"random character / reverb: max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL and min(xL, xR) == 1.0


def test_gpu_whirl_control_functions(oracle):
    """the whirl's MIDI control functions (src/whirl.cpp:699-889:
    horn filters A/B type, frequency, Q, gain; horn/drum brake positions; horn/drum
    acceleration and deceleration) through tbf_midi_control between renders, at seeded
    random values over the rotor stop -> fast -> stop -> slow -> stop script
    (scenarios.whirl_control_scenario: consecutive filter changes, out-of-range settings,
    a change while bypassed), against the oracle's orc_control.  The oracle's setter
    mapping equals the reference's own setters field for field (whirl.cpp built without
    CLAP, test_oracle_whirl_setters_pinned_to_reference), and the reference's whirlProc
    under those fields equals the oracle's (test_oracle_whirl_controls_vs_reference)."""
    n, nb = 8, 72
    eng, tpl, seeds, scens = _setup(oracle, n, S.whirl_control_scenario)
    L, R = engine_run(eng, scens, nb)
    oL, oR, *_ = oracle_run(oracle, tpl, seeds, scens, nb)
    eL, xL = compare(L, oL)
    eR, xR = compare(R, oR)
    print(f"whirl control functions: max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) == 0.0 and min(xL, xR) == 1.0
    eng.close()


@pytest.mark.parametrize("rate", [48000.0, 96000.0])
def test_gpu_whirl_split_kernel(oracle, rate):
    """k_whirl_split (two waves per instance: the horn and the drum halves of whirlProc2,
    dL / dR handed over in the drum rings' consumed slots) against k_whirl, bit for bit,
    over the whirl-control script (rotor stop / fast / brake / slow, filter and speed
    setters, a bypass toggle) at 48 kHz (ring of 512 samples) and 96 kHz (1024), with and
    without forced serial replays; and against the oracle.  (The engine picks k_whirl_split
    by itself at rings > 512 samples or <= 1 instance per CU, TBF_WHIRL_SPLIT=0 / 1 force
    either; most GPU tests here run small batches, so they run k_whirl_split.)"""
    import os
    import torch
    import tunebfree_amd as T
    n, nb = 24, 150
    seeds = [6100 + i for i in range(n)]
    scens = [S.whirl_control_scenario(i) for i in range(n)]
    for i in range(0, n, 5):
        scens[i] = sorted(scens[i] + [(90, "param", S.P_WHIRL_BYPASS, 1), (97, "param", S.P_WHIRL_BYPASS, 0)],
                          key=lambda r: r[0])
    outs = {}
    for split in ("0", "1"):
        for dbg in (0, 1):
            os.environ["TBF_WHIRL_SPLIT"] = split
            try:
                eng = T.Engine(sample_rate=rate, device=0, debug_flags=dbg)
            finally:
                os.environ.pop("TBF_WHIRL_SPLIT", None)
            tid = eng.template(seed=7)
            eng.add_instances([tid] * n, seeds)
            rows = []
            for i, sc in enumerate(scens):
                for (b, kind, a, v) in sc:
                    if kind == "note":
                        rows.append((b, i, 0, a, float(v)))
                    elif kind == "control":
                        rows.append((b, i, 2, eng.control_id(a), float(v)))
                    else:
                        rows.append((b, i, 1, a, float(v)))
            rows.sort(key=lambda r: r[0])
            L = torch.zeros((n, nb * 128), dtype=torch.float32, device="cuda")
            R = torch.zeros_like(L)
            eng.render_events_device(nb, eng.events(rows), L.data_ptr(), R.data_ptr(), nb * 128)
            eng.synchronize()
            outs[(split, dbg)] = (L.cpu().numpy(), R.cpu().numpy())
            eng.close()
            del L, R
    ref = outs[("0", 0)]
    for k, o in outs.items():
        assert np.array_equal(o[0].view(np.uint32), ref[0].view(np.uint32)), k
        assert np.array_equal(o[1].view(np.uint32), ref[1].view(np.uint32)), k
    if rate == 48000.0:
        from orc_bind import Template
        sample = [0, 5, 13, n - 1]
        tpl = Template(oracle, seed=7)
        oL, oR, *_ = oracle_run(oracle, tpl, [seeds[i] for i in sample], [scens[i] for i in sample], nb)
        eL, xL = compare(outs[("1", 0)][0][sample], oL)
        eR, xR = compare(outs[("1", 0)][1][sample], oR)
        print(f"k_whirl_split vs oracle: max|err| L={eL:.3g} R={eR:.3g} bit-exact {xL:.6f} {xR:.6f}")
        assert max(eL, eR) <= TOL


def test_gpu_whirl_control_events_threaded(oracle):
    """The same control functions as TBF_EV_CONTROL events inside one render of 72 blocks
    (across the 64-block chunk edge) for 1100 instances: the threaded host front end
    (stepChunkParallel: each worker's parameter sets rebased into the chunk's list) equals
    serial stepping bit for bit, and the oracle for instances from every worker's range."""
    import os
    import torch
    import tunebfree_amd as T
    from orc_bind import Template
    n, nb = 1100, 72
    seeds = [5000 + i for i in range(n)]
    scens = [S.whirl_control_scenario(i) for i in range(n)]
    outs = []
    for serial in (False, True):
        if serial:
            os.environ["TBF_HOST_SERIAL"] = "1"
        try:
            eng = T.Engine(sample_rate=48000.0, device=0)
        finally:
            os.environ.pop("TBF_HOST_SERIAL", None)
        tid = eng.template(seed=7)
        eng.add_instances([tid] * n, seeds)
        rows = []
        for i, sc in enumerate(scens):
            for (b, kind, a, v) in sc:
                if kind == "note":
                    rows.append((b, i, 0, a, float(v)))
                elif kind == "control":
                    rows.append((b, i, 2, eng.control_id(a), float(v)))
                else:
                    rows.append((b, i, 1, a, float(v)))
        ev = eng.events(rows)
        L = torch.zeros((n, nb * 128), dtype=torch.float32, device="cuda")
        R = torch.zeros_like(L)
        eng.render_events_device(nb, ev, L.data_ptr(), R.data_ptr(), nb * 128)
        eng.synchronize()
        outs.append((L.cpu().numpy(), R.cpu().numpy()))
        eng.close()
        del L, R
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1].view(np.uint32), outs[1][1].view(np.uint32))
    sample = [0, 1, 219, 220, 221, 440, 659, 660, 880, 1099]  # both sides of the 220-instance ranges
    tpl = Template(oracle, seed=7)
    oL, oR, *_ = oracle_run(oracle, tpl, [seeds[i] for i in sample], [scens[i] for i in sample], nb)
    eL, xL = compare(outs[0][0][sample], oL)
    eR, xR = compare(outs[0][1][sample], oR)
    print(f"whirl control events, threaded ({len(sample)} instances vs oracle): max|err| L={eL:.3g} R={eR:.3g}")
    assert max(eL, eR) == 0.0 and min(xL, xR) == 1.0


def _ring_window(max_ahead):
    """the compact whirl ring: the smallest of 512 / 1024 / 2048 holding the geometry's
    write-ahead + 2 + one 64-sample sub-block + 2 (tbf_engine.cpp buildShared)"""
    w = 512
    while w < max_ahead + 2 + 64 + 2:
        w *= 2
    return w


def test_gpu_cfg_widest_ring_96k(oracle):
    """The largest compact whirl ring (k_whirl<2048>): 96 kHz with an 80 cm horn, 4
    instances over the cfg script, against the oracle."""
    cfg = {"whirl.horn.radius": 80, "whirl.mic.distance": 60}
    eng, tpl, seeds, scens = _setup(oracle, 4, S.cfg_scenario, sr=96000.0, cfg=cfg)
    lay = eng.layout()
    assert lay["wring_len"] == _ring_window(lay["max_ahead"]) == 2048, lay
    L, R = engine_run(eng, scens, 72)
    oL, oR, *_ = oracle_run(oracle, tpl, seeds, scens, 72)
    eL, xL = compare(L, oL)
    eR, xR = compare(R, oR)
    print(f"96k / 2048-sample ring: max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL
    eng.close()


@pytest.mark.parametrize("name", sorted(S.CFG_SETS))
def test_gpu_cfg_keys(oracle, name):
    """§8(f) row 4: each cfg key set (scenarios.CFG_SETS — whirl geometry, the three
    whirl filters, speed preset + rpm + brake positions, horn/drum mic mix and widths,
    scanner rate/depths, reverb.mix, percussion gains/buses, the four envelope models)
    given to the engine through tbf_config_parse before its templates and instances,
    against the oracle under the same orc_cfg (itself bit-identical to the reference's
    own structs, test_oracle_cpu.py::test_oracle_cfg_vs_reference): every stage tap,
    6 instances over the rotor stop -> fast -> brake -> slow script."""
    n, nb = 6, 72
    eng, tpl, seeds, scens = _setup(oracle, n, S.cfg_scenario, cfg=S.CFG_SETS[name])
    lay = eng.layout()
    assert lay["wring_len"] == _ring_window(lay["max_ahead"]) == (1024 if name == "geometry_wide" else 512), lay
    L, R = engine_run(eng, scens, nb)
    oL, oR, oA, oB, oC = oracle_run(oracle, tpl, seeds, scens, nb)
    eL, xL = compare(L, oL)
    eR, xR = compare(R, oR)
    print(f"cfg {name}: max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL
    for i in range(n):
        assert float(np.abs(oL[i]).max()) > 1e-3
    eng.close()


def test_gpu_retune_mid_phrase(oracle, tunings):
    """§8(f) row 3, the MTS-ESP retune (tbf_instance_retune = the CLAP reinitToneGen,
    src/clap.cpp:129-157): 6 instances switch mid-phrase to a 19-TET template built on
    the device (tbf_templates_create) and later back to their 12-TET template; held keys
    drop, drawbars / vibrato come back from the CLAP parameters (their defaults where
    never set), the routing word stays, preamp / reverb / whirl state goes on.  Against
    the oracle's orc_inst_retune (itself bit-identical to the reference's own calls,
    test_oracle_cpu.py::test_oracle_retune_vs_reference), every stage tap."""
    from orc_bind import Template
    m19 = np.asarray(tunings["19TET"], np.float64)
    n, nb = 6, 64
    eng = _engine()
    tid12 = eng.template(seed=7)
    tid19 = eng.templates([8], mts128=m19[None])[0]
    seeds = [1000 + 17 * i for i in range(n)]
    eng.add_instances([tid12] * n, seeds)
    t12, t19 = Template(oracle, seed=7), Template(oracle, mts128=m19, seed=8)
    scens = [S.retune_scenario(i, at=20, to=1) + [(44, "retune", 0, 0), (44, "note", 62 + i, 1)] for i in range(n)]
    L, R = engine_run(eng, scens, nb, tids=[tid12, tid19])
    oL, oR, *_ = oracle_run(oracle, t12, seeds, scens, nb, templates=[t12, t19])
    eL, xL = compare(L, oL)
    eR, xR = compare(R, oR)
    print(f"retune: max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL
    for i in range(n):
        assert float(np.abs(oL[i, 21 * 128:44 * 128]).max()) > 1e-3  # the retuned organ sounds
    eng.close()


@pytest.mark.parametrize("scen", ["events", "sweep", "reroute", "retune"])
def test_gpu_device_control_programs(oracle, tunings, scen):
    """§8(f) row 1: the per-wheel control on the device (k_tgctl: message queue ->
    activated-oscillator table -> active list -> routed sums -> core program) emits, block
    by block, the oracle's oscGenerateFragment programs (wheel order, envelope rows, all
    six gains bit for bit), read back from the device's program pool after each
    one-block render."""
    import ctypes as C
    import tunebfree_amd as T
    from orc_bind import Chain, Template
    from test_host_cpu import _events_by_block, _oracle_program, _orc_bind_debug
    _orc_bind_debug(oracle)
    lib = T.load_library()
    fn = lib.tbf_debug_device_program
    fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]
    m19 = np.asarray(tunings["19TET"], np.float64)
    eng = _engine()
    tpls = [Template(oracle, seed=7), Template(oracle, mts128=m19, seed=8)]
    tids = [eng.template(seed=7), eng.template(mts128=m19, seed=8)]
    n_inst, nblocks = 3, 56
    seeds = [1000 + i for i in range(n_inst)]
    eng.add_instances([tids[0]] * n_inst, seeds)
    chains = [Chain(oracle, tpls[0], sd) for sd in seeds]
    gen = {"events": S.event_scenario, "sweep": S.sweep_scenario, "reroute": S.reroute_scenario,
           "retune": lambda i: S.retune_scenario(i, at=20, to=1) + [(44, "retune", 0, 0), (44, "note", 62, 1)]}[scen]
    scens = [_events_by_block(gen(i)) for i in range(n_inst)]
    buf = np.zeros(9 * 600, np.float32)
    checked = 0
    for blk in range(nblocks):
        for i in range(n_inst):
            for (kind, a, v) in scens[i].get(blk, []):
                if kind == "note":
                    eng.note(i, a, v)
                    chains[i].note(a, v)
                elif kind == "retune":
                    eng.retune(i, tids[a])
                    chains[i].retune(tpls[a])
                else:
                    eng.set_param(i, a, v)
                    chains[i].param(a, v)
            chains[i].render(1)
        eng.render(1)
        for i in range(n_inst):
            op = _oracle_program(oracle, chains[i].ptr)
            n = fn(eng._h, i, buf.ctypes.data, 600)
            assert n == len(op), (blk, i, n, len(op))
            pp = buf[: 9 * n].reshape(n, 9)
            for (w, env, r, g), q in zip(op, pp):
                assert (w, env) == (int(q[0]), int(q[1])), (blk, i)
                if env:
                    assert r == int(q[2]), (blk, i)
                    assert np.array_equal(g.view(np.uint32), q[3:9].view(np.uint32)), (blk, i, w)
                else:
                    assert np.array_equal(g[:3].view(np.uint32), q[3:6].view(np.uint32)), (blk, i, w)
                checked += 1
    print(f"device control programs ({scen}): {checked} instructions bit-exact")
    assert checked > 500
    eng.close()


def test_gpu_device_control_large_clusters(oracle):
    """k_tgctl's paths past its fast ones (tbf_ctl.hip): 12-key clusters released and
    pressed on every block put 24 messages in a block and ~1500 in a 64-block launch (more
    than the CTL_MSGCAP prefetched into LDS: read per block), a key's passes over its
    keyContrib list in groups, active lists over 64 wheels (a second pass of the active-list
    loop, its removals through LDS) and more than 64 wheels leaving at once (the serial
    removal loop); lighter instances in the same launch keep the fast paths.  Device front
    end, host front end (TBF_DEVICE_FRONT=0) and host control (TBF_HOST_CONTROL=1, no
    k_tgctl) bit-identical, and the oracle for a sample."""
    import os
    import torch
    import tunebfree_amd as T
    from orc_bind import Template
    n, nb = 48, 128
    seeds = [8100 + i for i in range(n)]
    rows, oscen = [], [[] for _ in range(n)]

    def ev(b, i, kind, a, v):
        rows.append((b, i, 0 if kind == "note" else 1, a, float(v)))
        oscen[i].append((b, kind, a, v))

    def cluster(i, t):
        base = 36 + (3 * i + 5 * t) % 40
        return [base + 2 * k for k in range(12)]

    for i in range(n):
        for (k, a, v) in S.jazz1_params():
            ev(0, i, k, a, v)
        heavy = i % 3 != 2
        cur = cluster(i, 0) if heavy else S.chord_for(i)
        for k in cur:
            ev(0, i, "note", k, 1)
        for b in range(1, nb):
            if heavy:
                if b % 16 == 15:  # everything released: over 64 wheels leave in one block
                    for k in cur:
                        ev(b, i, "note", k, 0)
                    cur = []
                    continue
                nxt = cluster(i, b)
                for k in cur:
                    ev(b, i, "note", k, 0)
                for k in nxt:
                    ev(b, i, "note", k, 1)
                cur = nxt
            else:
                ev(b, i, "note", 60 + (i + b - 1) % 12, 0)
                ev(b, i, "note", 60 + (i + b) % 12, 1)
    rows.sort(key=lambda r: r[0])
    outs = []
    for env in ({}, {"TBF_DEVICE_FRONT": "0"}, {"TBF_HOST_CONTROL": "1"}):
        os.environ.update(env)
        try:
            eng = T.Engine(sample_rate=48000.0, device=0)
        finally:
            for k in env:
                os.environ.pop(k, None)
        tid = eng.template(seed=7)
        eng.add_instances([tid] * n, seeds)
        evs = eng.events(rows)
        L = torch.zeros((n, nb * 128), dtype=torch.float32, device="cuda")
        R = torch.zeros_like(L)
        eng.render_events_device(nb, evs, L.data_ptr(), R.data_ptr(), nb * 128)
        eng.synchronize()
        outs.append((L.cpu().numpy(), R.cpu().numpy()))
        eng.close()
        del L, R
    for o in outs[1:]:
        assert np.array_equal(outs[0][0].view(np.uint32), o[0].view(np.uint32))
        assert np.array_equal(outs[0][1].view(np.uint32), o[1].view(np.uint32))
    sample = [0, 1, 2, 29]
    tpl = Template(oracle, seed=7)
    oL, oR, *_ = oracle_run(oracle, tpl, [seeds[i] for i in sample], [sorted(oscen[i], key=lambda r: r[0]) for i in sample], nb)
    eL, xL = compare(outs[0][0][sample], oL)
    eR, xR = compare(outs[0][1][sample], oR)
    print(f"large clusters vs oracle: max|err| L={eL:.3g} R={eR:.3g} bit-exact {xL:.6f} {xR:.6f}")
    assert max(eL, eR) <= TOL


def test_gpu_reroute_without_key_events(oracle):
    """Drawbar / vibrato-routing / percussion changes while keys are held, with no key
    event in the block (scenarios.reroute_scenario): the new sums must take effect from
    the next block, as in the reference (the render path steps the control plane only
    when something changed)."""
    eng, tpl, seeds, scens = _setup(oracle, 4, S.reroute_scenario)
    L, R = engine_run(eng, scens, 56)
    oL, oR, *_ = oracle_run(oracle, tpl, seeds, scens, 56)
    eL, xL = compare(L, oL)
    eR, xR = compare(R, oR)
    print(f"reroute: max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL


def test_gpu_forced_serial_events_and_taps(oracle):
    """The event script (chord changes, note-offs with release envelopes, lower-manual
    vibrato, rotary fast -> slow) and the preamp / reverb stage taps with every guarded
    stage on its serial replay."""
    eng, tpl, seeds, scens = _setup(oracle, 4, S.event_scenario, debug_flags=1)
    L, R = engine_run(eng, scens, 72)
    oL, oR, *_ = oracle_run(oracle, tpl, seeds, scens, 72)
    eL, xL = compare(L, oL)
    eR, xR = compare(R, oR)
    print(f"forced events: max|err| L={eL:.3g} R={eR:.3g} bit-exact L={xL:.6f} R={xR:.6f}")
    assert max(eL, eR) <= TOL
    for tap, idx in ((2, 3), (3, 4)):
        eng, tpl, seeds, scens = _setup(oracle, 3, S.sweep_scenario, chain=tap, debug_flags=1)
        L, _ = engine_run(eng, scens, 40)
        ref = oracle_run(oracle, tpl, seeds, scens, 40)[idx]
        err, exact = compare(L, ref)
        print(f"forced tap {tap}: max|err|={err:.3g} bit-exact={exact:.6f}")
        assert err <= TOL


@pytest.mark.parametrize("via_events", [True, False])
def test_gpu_add_instances_after_render_then_events(oracle, via_events):
    """Instances added to an engine that has already rendered; then one
    tbf_render_events call with events at blocks > 0 for instances that existed before
    (and for new ones): an old instance's blocks before its event must still render with
    its earlier control (the persistent control pool is uploaded as of the chunk start)."""
    import torch
    from orc_bind import Template
    eng = _engine()
    tid = eng.template(seed=7)
    seeds = [1000 + 17 * i for i in range(5)]
    eng.add_instances([tid] * 3, seeds[:3])
    pre = [S.bench_scenario(i) for i in range(3)]
    L0, R0 = engine_run(eng, pre, 10)
    eng.add_instances([tid] * 2, seeds[3:])
    for i in (3, 4):
        for (b, kind, a, v) in S.bench_scenario(i):
            (eng.note if kind == "note" else eng.set_param)(i, a, v)
    nb = 40
    rows = [(5, 0, 0, 72, 1.0), (5, 0, 1, S.P_HORN, 2.0), (9, 1, 1, S.P_DRAWBAR + 4, 7.0),
            (17, 2, 0, 60 + 2, 0.0), (20, 2, 1, S.P_REVERB, 0.6), (7, 4, 0, 50, 1.0), (30, 1, 1, S.P_CHARACTER, 0.9)]
    if via_events:
        L = torch.zeros((5, nb * 128), dtype=torch.float32, device="cuda")
        R = torch.zeros_like(L)
        eng.render_events_device(nb, eng.events(rows), L.data_ptr(), R.data_ptr(), nb * 128)
        eng.synchronize()
        L, R = L.cpu().numpy(), R.cpu().numpy()
    else:  # the same script through tbf_note / tbf_set_param between render calls
        sc5 = [[(b, "note" if k == 0 else "param", a, v) for (b, inst, k, a, v) in rows if inst == i]
               for i in range(5)]
        L, R = engine_run(eng, sc5, nb)
    tpl = Template(oracle, seed=7)
    bad = []
    for i in range(5):
        off = 10 if i < 3 else 0  # old instances: the call starts at their block 10
        sc = list(S.bench_scenario(i))
        for (b, inst, kind, a, v) in rows:
            if inst == i:
                sc.append((b + off, "note" if kind == 0 else "param", a, v))
        oL, oR, *_ = oracle_run(oracle, tpl, [seeds[i]], [sc], nb + off)
        gl = np.concatenate([L0[i], L[i]]) if off else L[i]
        gr = np.concatenate([R0[i], R[i]]) if off else R[i]
        e1, x1 = compare(gl, oL[0])
        e2, x2 = compare(gr, oR[0])
        d = np.nonzero(gl.view(np.uint32) != oL[0].view(np.uint32))[0]
        print(f"instance {i}: max|err| {max(e1, e2):.3g} bit-exact {min(x1, x2):.6f} "
              f"first differing block {d[0] // 128 if len(d) else None}")
        if max(e1, e2) > TOL:
            bad.append(i)
    assert not bad, bad


def test_gpu_sin_fast_paths_are_ocml_bits():
    """csrc/tbf_sin.h: the kernels' sin with wave-uniform fast paths (only the sine or only
    the cosine polynomial of OCML's reduction when every lane of a wave has n = 0 or n = 1,
    OCML's small-argument path inline otherwise), the paired tbf_sin2 and the asin polynomial
    branch return the device library's sin / asin bit for bit: sorted inputs (uniform waves on both fast
    paths), shuffled ones (mixed waves: the library path), negatives, the n = 0 / 1 / 2
    boundaries, the preamp's clamp 1.57079633, signed zeros, subnormals, huge values
    (Payne-Hanek), infinities and NaN (through tbf_debug_calibrate op 4)."""
    import ctypes as C
    import torch
    import tunebfree_amd as T
    lib = T.load_library()
    lib.tbf_debug_calibrate.restype = C.c_int
    lib.tbf_debug_calibrate.argtypes = [C.c_int32, C.c_void_p, C.c_uint64, C.c_void_p]
    rng = np.random.default_rng(5)
    q = np.pi / 4
    sorted_ = np.sort(rng.uniform(0.0, 1.6, 1 << 18))
    mixed = rng.permutation(sorted_)
    edges = np.concatenate([np.nextafter(q, 0) - np.arange(64) * 1e-16, q + np.arange(64) * 1e-16,
                            3 * q + np.arange(-64, 64) * 1e-16, np.full(64, 1.57079633),
                            np.full(64, 0.0), np.full(64, -0.0), np.full(64, 5e-324), np.full(64, 1e-300)])
    special = np.array([np.inf, -np.inf, np.nan, 1e300, -1e22, 2.0 ** 30, -(2.0 ** 30) + 1, 1e9, 3.0, -2.5] * 7,
                       dtype=np.float64)
    x = np.concatenate([sorted_, -sorted_, mixed, edges, special, rng.normal(0, 0.05, 1 << 16)])
    n = len(x)
    buf = torch.zeros(7 * n, dtype=torch.float64, device="cuda")
    buf[:n] = torch.from_numpy(x).cuda()
    assert lib.tbf_debug_calibrate(4, C.c_void_p(buf.data_ptr()), n, None) == 0
    torch.cuda.synchronize()
    out = buf.cpu().numpy().reshape(7, n)
    ref = out[2]
    other = np.roll(ref, -(n // 2))  # sin of the input n / 2 further on
    for name, got, want in (("tbf_sin", out[1], ref), ("tbf_sin2 first", out[3], ref),
                            ("tbf_sin2 second", out[4], other), ("asin fast path", out[5], out[6])):
        same = got.view(np.uint64) == want.view(np.uint64)
        assert same.all(), (name, x[~same][:8], got[~same][:8], want[~same][:8])
    assert np.mean(np.abs(np.clip(x, -1, 1)) < 0.5) > 0.3  # the asin fast path was exercised
