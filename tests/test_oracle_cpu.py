"""CPU tests: pin the oracle to the reference's own fixtures and known answers, and
(where /root/reference is present) to the reference's compiled translation units.

Fixture provenance (tests/golden/make_fixtures.py):
  - regression_test_data.tar.xz: the reference's tests/regression_test_data (the
    DEBUG_TONEGEN_OSC dumps compared by tests/test_regression.py in the reference);
  - tunings.json: the frequency tables the reference's doctests embed
    (src/tuning.cpp:208-395) and the two .scl-defined sets.
"""
import ctypes as C
import json
import re
import tarfile
from pathlib import Path

import numpy as np
import pytest

import scenarios as S
from orc_bind import Chain, Template, fptr

GOLD = Path(__file__).resolve().parent / "golden"
SETS = ["12TET", "19TET", "5TET", "bagpipe4", "duodene", "p4"]


@pytest.fixture(scope="module")
def fixtures(tmp_path_factory):
    d = tmp_path_factory.mktemp("regr")
    with tarfile.open(GOLD / "regression_test_data.tar.xz") as tf:
        tf.extractall(d)
    return d / "regression_test_data"


def test_rand_is_glibc_rand(oracle):
    """orc_rand == the C library's rand() after srand(seed) (TYPE_3, glibc)."""
    libc = C.CDLL(None)
    st = C.create_string_buffer(256)
    for seed in (1, 7, 12345, 0, 4294967295):
        libc.srand(C.c_uint(seed))
        a = [libc.rand() for _ in range(3000)]
        oracle.orc_srand(st, seed)
        b = [oracle.orc_rand_next(st) for _ in range(3000)]
        assert a == b, seed


def test_fitwave_known_answers(oracle):
    """src/tonegen.cpp:4176-4222 doctest values (TEST_RATE 48000)."""
    mc = 440 * 2.0 ** (-9.0 / 12.0)
    n = 1000000000
    fw = lambda hz, p, lo, hi: oracle.orc_fitwave(hz, p, lo, hi, 48000.0)
    assert [fw(mc, p, 1, n) for p in (0.0001, 0.001, 0.01, 0.1, 1.0)] == [610766, 52105, 14494, 367, 183]
    assert [fw(mc, p, 384, 4096) for p in (0.0001, 0.001, 0.01, 0.1, 1.0)] == [2752, 2752, 2752, 2385, 550]
    mult = [1 / 32, 1 / 16, 1 / 8, 1 / 4, 1 / 2, 1, 2, 4, 8, 16, 32]
    assert [fw(mc * m, 0.001, 1, n) for m in mult] == [2495169, 2286749, 104210, 52105, 52105, 52105, 52105,
                                                       22429, 14838, 7419, 86]
    assert [fw(mc * m, 0.001, 384, 4096) for m in mult[1:]] == [2935, 1468, 734, 734, 2752, 1376, 688, 688, 516, 430]


def test_frequencies_known_answers(oracle):
    """src/tuning.cpp:178-206 getMTSESPFrequencies / extendFrequencies / getFrequencies."""
    f = np.zeros(300)
    oracle.orc_get_frequencies(f.ctypes.data_as(C.POINTER(C.c_double)), None)
    assert f[0] == 8.1757989156437070
    assert f[24] == 32.70319566257483 and f[36] == 2 * 32.70319566257483
    assert f[114] == 5919.91076338615039 and f[102] == 5919.91076338615039 / 2
    assert f[128] == 13289.75032255824408 and f[255] == 20390018.00521029531956


@pytest.mark.parametrize("name,size,period", [("19TET", 19, 2.0), ("Bohlen-Pierce", 13, 3.0), ("p4", 4, 7.0),
                                              ("bagpipe4", 9, 1.9884808063507080)])
def test_infer_scale_size(oracle, tunings, name, size, period):
    """src/tuning.cpp:208-395 inferPeriod doctests."""
    f = np.array(tunings[name], np.float64)
    s, p = C.c_int(), C.c_float()
    oracle.orc_infer_scale_size(f.ctypes.data_as(C.POINTER(C.c_double)), C.byref(s), C.byref(p))
    assert s.value == size and p.value == np.float32(period)


def test_extend_bagpipe4(oracle, tunings):
    """src/tuning.cpp:397-435: extension beyond 128 notes with a 1190-cent period."""
    f = np.zeros(300)
    m = np.array(tunings["bagpipe4"], np.float64)
    oracle.orc_get_frequencies(f.ctypes.data_as(C.POINTER(C.c_double)), m.ctypes.data)
    assert f[128] == 42881.3840096949352301 and f[255] == 728988980.0540838241577148


_ENTRY = re.compile(r"\[w\s*(\d+):b\s*(\d+):g([0-9.]+)\]\s+(-?[0-9.]+) dB  (I*)$")


@pytest.mark.parametrize("name", SETS)
def test_regression_fixtures(oracle, fixtures, tunings, name, tmp_path):
    """The reference's tests/test_regression.py fixtures: osc.txt and osc_cfglists.txt
    byte-identical; osc_runtime.txt identical in every wheel, bus, gain (%f), bar and
    count, with the dB column within 1e-5 (the fixtures were produced by the
    reference's -ffast-math release build, whose crosstalk gains differ from a strict
    build in the last float bits -- see DESIGN.md)."""
    m = tunings[name]
    t = Template(oracle, mts128=None if m is None else np.array(m))
    assert t.dump(tmp_path) == 0
    for fn in ("osc.txt", "osc_cfglists.txt"):
        assert (tmp_path / fn).read_bytes() == (fixtures / name / fn).read_bytes(), fn
    a = (tmp_path / "osc_runtime.txt").read_text().splitlines()
    b = (fixtures / name / "osc_runtime.txt").read_text().splitlines()
    assert len(a) == len(b)
    worst = 0.0
    for x, y in zip(a, b):
        if x == y:
            continue
        mx, my = _ENTRY.search(x), _ENTRY.search(y)
        assert mx and my, (x, y)
        assert mx.group(1, 2, 3, 5) == my.group(1, 2, 3, 5), (x, y)
        assert x[:x.index("]")] == y[:y.index("]")]
        worst = max(worst, abs(float(mx.group(4)) - float(my.group(4))))
    assert worst <= 1e-5


# --------------------------------------------------------------------------- reference TUs
def test_oracle_chain_bitexact_vs_reference(oracle, refchk):
    """Full quartet (tonegen+vibrato -> density -> MatrixVerb -> whirlProc3) of the
    oracle vs the reference's own compiled code on identical inputs, all stages."""
    tpl = Template(oracle, seed=7)
    for scen, nb in ((S.bench_scenario(3), 48), (S.event_scenario(5), 72)):
        a = Chain(oracle, tpl, 11)
        b = Chain(refchk, tpl, 11, ref=True)
        oa = S.run(a, scen, nb, stages=True)
        ob = S.run(b, scen, nb, stages=True)
        for x, y in zip(oa, ob):
            assert np.array_equal(x.view(np.uint32), y.view(np.uint32))


def test_oracle_tonegen_only_vs_reference(oracle, refchk):
    tpl = Template(oracle, seed=3)
    for i in range(3):
        sc = S.bench_scenario(i, full=False) + [(20, "note", 70, 1), (30, "param", S.P_PERC, 1)]
        a = Chain(oracle, tpl, 5 + i)
        b = Chain(refchk, tpl, 5 + i, ref=True)
        a.chain(1)
        b.chain(1)
        x = S.run(a, sc, 40, stages=True)[2]
        y = S.run(b, sc, 40, stages=True)[2]
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))


@pytest.mark.parametrize("sr", [44100.0, 48000.0, 96000.0])
def test_stage_units_vs_reference(oracle, refchk, sr):
    """Each effect stage alone on seeded noise + impulses + silence (denormal path)."""
    rng = np.random.default_rng(int(sr))
    n = 128 * 40
    x = (rng.standard_normal(n) * 0.3).astype(np.float32)
    x[1000:1300] = 0.0
    x[2000] = 1.5
    for opt in (4, 8, 0, 2):
        wo, wr = oracle.orc_whirl_new(sr), refchk.ref_whirl_new(sr)
        oracle.orc_whirl_rev_option(wo, opt)
        refchk.ref_whirl_rev_option(wr, opt)
        a = [np.zeros(n, np.float32) for _ in range(4)]
        oracle.orc_whirl_proc3(wo, fptr(x), fptr(a[0]), fptr(a[1]), 128 * 20)
        refchk.ref_whirl_proc3(wr, fptr(x), fptr(a[2]), fptr(a[3]), 128 * 20)
        assert np.array_equal(a[0].view(np.uint32), a[2].view(np.uint32))
        assert np.array_equal(a[1].view(np.uint32), a[3].view(np.uint32))
        oracle.orc_whirl_free(wo)
        refchk.ref_whirl_free(wr)
    for seed in (1, 99):
        ro, rr = oracle.orc_reverb_new(sr, seed), refchk.ref_reverb_new(sr, seed)
        for g in (0.1, 0.7):
            oracle.orc_reverb_set_mix(ro, g)
            refchk.ref_reverb_set_mix(rr, g)
            a, b = np.zeros(n, np.float32), np.zeros(n, np.float32)
            oracle.orc_reverb_proc(ro, fptr(x), fptr(a), n)
            refchk.ref_reverb_proc(rr, fptr(x), fptr(b), n)
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
        oracle.orc_reverb_free(ro)
        refchk.ref_reverb_free(rr)
    for ch in (0.0, 0.3, 0.5, 0.9, 1.0):
        po, pr = oracle.orc_preamp_new(sr, 5), refchk.ref_preamp_new(sr, 5)
        oracle.orc_preamp_set(po, 0, ch)
        refchk.ref_preamp_set(pr, 0, ch)
        a, b = np.zeros(n, np.float32), np.zeros(n, np.float32)
        oracle.orc_preamp_proc(po, fptr(x), fptr(a), n)
        refchk.ref_preamp_proc(pr, fptr(x), fptr(b), n)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
        oracle.orc_preamp_free(po)
        refchk.ref_preamp_free(pr)


# --------------------------------------------------------------------------- committed vectors
def _golden_cases():
    z = np.load(GOLD / "ref_vectors.npz")
    return z, json.loads(str(z["cases"]))


def test_glibc_rand_python_mirror():
    """scenarios.GlibcRand (used by the config-5 random-drawbar scripts) == libc rand()."""
    libc = C.CDLL(None)
    for seed in (1, 3, 12345, 0, 2 ** 31 + 5):
        libc.srand(C.c_uint(seed))
        a = [libc.rand() for _ in range(500)]
        g = S.GlibcRand(seed)
        assert a == [g.next() for _ in range(500)], seed


def test_oracle_vs_committed_reference_vectors(oracle, tunings):
    """The oracle reproduces, bit for bit and at every stage tap, the outputs of the
    reference's own compiled TUs committed in tests/golden/ref_vectors.npz (generator:
    tests/golden/make_ref_vectors.py) -- 44.1/48/96 kHz, 4 tunings, event scripts."""
    from golden.make_ref_vectors import scenario
    z, cases = _golden_cases()
    assert len(cases) >= 6
    for c in cases:
        m = None if c["tuning"] is None else np.array(tunings[c["tuning"]], np.float64)
        tpl = Template(oracle, sr=c["sr"], mts128=m, seed=c["tpl_seed"])
        ch = Chain(oracle, tpl, c["inst_seed"])
        ch.chain(c["chain"])
        got = S.run(ch, scenario(*c["scenario"]), c["nblocks"], stages=True)
        for k, v in zip("LRABC", got):
            ref = z[f"{c['name']}/{k}"]
            assert np.array_equal(v.view(np.uint32), ref.view(np.uint32)), (c["name"], k)


# --------------------------------------------------------------------------- template pins
def _template_pins():
    return json.loads((GOLD / "template_pins.json").read_text())


def test_oracle_templates_vs_reference_pins(oracle, tunings):
    """The oracle's wave banks (writeSamples sines + per-sample rand() LSB), wheel
    lengths, envelopes, key-compression tables and play matrices equal, bit for bit, the
    tables the reference's own src/tonegen.cpp builds (static initOscillators /
    initKeyCompTable / initEnvelopes / applyManualDefaults / compilePlayMatrix ... reached
    by oracle/ref_tpl_pin.cpp; digests committed in tests/golden/template_pins.json by
    tests/golden/make_template_pins.py): 7 tunings x 48 / 96 kHz, plus the osc.* cfg sets
    (envelope models, wheel EQ, harmonics, terminal / taper / crosstalk lists)."""
    import hashlib
    from orc_bind import Cfg
    pins = _template_pins()
    assert len(pins) == 19
    for p in pins:
        m = None if tunings[p["tuning"]] is None else np.array(tunings[p["tuning"]], np.float64)
        cfg = Cfg(oracle, S.CFG_SETS[p["cfg"]]) if p.get("cfg") else None
        tpl = Template(oracle, sr=p["sr"], mts128=m, seed=p["seed"], cfg=cfg)
        bank, lens = tpl.bank()
        a, r, k = tpl.envs()
        got = {"bank": bank, "lens": lens, "attack": a, "release": r, "keycomp": k, "contrib": tpl.contrib()}
        for key, v in got.items():
            assert hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest() == p[key], \
                (p["tuning"], p["sr"], p.get("cfg"), key)


def test_reference_pin_harness_reproduces_committed_pins(oracle, tunings):
    """Where /root/reference is built (oracle/_ref/libtbfpin.so), the reference's own
    builders still give the committed digests (the fixture is current)."""
    from golden.make_template_pins import cases, digest
    from orc_bind import Cfg, load_pin, pin_template
    pin = load_pin()
    if pin is None:
        pytest.skip("oracle/_ref/libtbfpin.so not built (no /root/reference here)")
    pins = _template_pins()
    meta = ("tuning", "sr", "seed", "cfg")
    for (nm, sr, seed, m, cfgname), p in zip(cases(), pins):
        cfg = Cfg(oracle, S.CFG_SETS[cfgname]) if cfgname else None
        d = digest(pin_template(pin, oracle, sr, m, seed, cfg))
        assert {k: d[k] for k in p if k not in meta} == {k: p[k] for k in p if k not in meta}, (nm, sr, cfgname)


# --------------------------------------------------------------------------- cfg keys
@pytest.mark.parametrize("name", sorted(S.CFG_SETS))
def test_oracle_cfg_vs_reference(oracle, refchk, name):
    """Each cfg key set (scenarios.CFG_SETS: whirl geometry, filters, speeds + brake
    positions, mic mix / scanner / reverb.mix / percussion, envelope models) applied by
    the oracle (orc_cfg_set) and, on the reference's own structs, by the harness: the
    chain is bit-identical at every stage tap over a rotor stop -> fast -> brake -> slow
    script."""
    from orc_bind import Cfg
    cfg = Cfg(oracle, S.CFG_SETS[name])
    tpl = Template(oracle, sr=48000.0, seed=7, cfg=cfg)
    for i in range(2):
        sc = S.cfg_scenario(i)
        a = S.run(Chain(oracle, tpl, 500 + i), sc, 72, stages=True)
        b = S.run(Chain(refchk, tpl, 500 + i, ref=True), sc, 72, stages=True)
        for k, x, y in zip("LRABC", a, b):
            assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), (name, i, k)
        assert float(np.abs(a[0]).max()) > 1e-3


def test_oracle_whirl_controls_vs_reference(oracle, refchk):
    """the whirl's MIDI control functions (horn filters, brake
    positions, ramp times; src/whirl.cpp:699-889) mid-run.  The oracle (orc_control) and
    the harness (ref_control: the reference's struct fields and its own eqCompute; the
    setters themselves are compiled out under the CLAP define) feed the reference's own
    whirlProc2/3, bit-identical at every stage tap over the rotor script."""
    tpl = Template(oracle, sr=48000.0, seed=7)
    for i in range(4):
        sc = S.whirl_control_scenario(i)
        a = S.run(Chain(oracle, tpl, 700 + i), sc, 72, stages=True)
        b = S.run(Chain(refchk, tpl, 700 + i, ref=True), sc, 72, stages=True)
        for k, x, y in zip("LRABC", a, b):
            assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), (i, k)
        # the controls change the output (against the same script without them)
        c = S.run(Chain(oracle, tpl, 700 + i), [e for e in sc if e[1] != "control"], 72)
        assert not np.array_equal(a[0], c[0])


def test_oracle_whirl_setters_pinned_to_reference(oracle):
    """The whirl's MIDI control setters (src/whirl.cpp:699-909) pinned to the reference's
    own functions: oracle/ref_whirl_pin.cpp #includes whirl.cpp without the CLAP define
    and calls its static setters by the names initWhirl registers (970-981).  Over every
    function x every value 0..127 at three rates, and a seeded random sequence of
    controls, the fields each setter writes (filter type / Hz / Q / gain with the
    recomputed biquad after setIIRFilter's range guard, brake positions, ramp rates)
    equal the oracle's orc_control's field for field."""
    from orc_bind import load_wpin
    wp = load_wpin()
    if wp is None:
        pytest.skip("oracle/_ref/libtbfwpin.so not built (no /root/reference here)")
    tpl = Template(oracle, sr=48000.0, seed=7)

    def fields(getter, h):
        out = np.zeros(24, np.float64)
        assert getter(h, out.ctypes.data_as(C.POINTER(C.c_double))) == 24
        return out

    rng = np.random.default_rng(5)
    for sr in (44100.0, 48000.0, 96000.0):
        t = tpl if sr == 48000.0 else Template(oracle, sr=sr, seed=7)
        ch = Chain(oracle, t, 1)
        w = wp.wpin_new(sr)
        try:
            assert np.array_equal(fields(oracle.orc_whirl_fields, ch.ptr), fields(wp.wpin_fields, w)), sr
            script = [(n, v) for n in S.WHIRL_CONTROLS for v in range(128)]
            script += [(S.WHIRL_CONTROLS[int(rng.integers(len(S.WHIRL_CONTROLS)))], int(rng.integers(128)))
                       for _ in range(2000)]
            for name, v in script:
                ch.control(name, v)
                assert wp.wpin_control(w, name.encode(), v) == 0
                a, b = fields(oracle.orc_whirl_fields, ch.ptr), fields(wp.wpin_fields, w)
                assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), (sr, name, v, a, b)
            assert wp.wpin_control(w, b"rotary.speed-toggle", 1) == -1
        finally:
            wp.wpin_free(w)


def test_oracle_whirl_control_names(oracle):
    """orc_control knows exactly the 14 functions initWhirl registers (966-981)."""
    tpl = Template(oracle, sr=48000.0, seed=7)
    ch = Chain(oracle, tpl, 1)
    for name in S.WHIRL_CONTROLS:
        ch.control(name, 64)
    for bad in ("whirl.horn.filter.c.type", "whirl.drum.filter.hz", "rotary.speed-toggle", "whirl.horn.brakepos "):
        with pytest.raises(ValueError):
            ch.control(bad, 1)


def test_oracle_cfg_parsing(oracle):
    """orc_cfg_set follows getConfigParameter_*: ranges are inclusive, a bad or
    out-of-range value assigns nothing (-1), unknown keys are ignored (0)."""
    from orc_bind import Cfg
    c = Cfg(oracle)
    assert c.set("whirl.horn.brakepos", "0.5") == 1
    assert c.set("whirl.horn.brakepos", "1.5") == -1
    assert c.set("whirl.drum.filter.type", "9") == -1
    assert c.set("scanner.hz", "3.9") == -1 and c.set("scanner.hz", "4") == 1
    assert c.set("WHIRL.HORN.RADIUS", "20") == 1  # strcasecmp
    assert c.set("midi.upper.channel", "1") == 0


# --------------------------------------------------------------------------- retune
def test_oracle_retune_vs_reference(oracle, refchk, tunings):
    """§8(f) row 3, the MTS-ESP retune: the CLAP plugin's reinitToneGen
    (src/clap.cpp:129-157) on a new template mid-phrase -- the oracle (orc_inst_retune)
    against the reference's own calls (ref_inst_retune: allocTonegen tables,
    init_vibrato, setDrawBar / setVibratoUpper / setVibratoFromInt from the parameters,
    newRouting kept), bit for bit at every stage tap; 4 variants (parameters set / at
    their CLAP defaults, percussion on / off) and retunes to 19-TET and back to 12-TET."""
    t12 = Template(oracle, sr=48000.0, seed=7)
    t19 = Template(oracle, sr=48000.0, mts128=np.array(tunings["19TET"], np.float64), seed=8)
    for i in range(4):
        sc = S.retune_scenario(i, at=20, to=1) + [(40, "retune", 0, 0), (41, "note", 60 + i, 1)]
        a = S.run(Chain(oracle, t12, 600 + i), sc, 56, stages=True, templates=[t12, t19])
        b = S.run(Chain(refchk, t12, 600 + i, ref=True), sc, 56, stages=True, templates=[t12, t19])
        for k, x, y in zip("LRABC", a, b):
            assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), (i, k)
        assert float(np.abs(a[0][21 * 128:]).max()) > 1e-3
