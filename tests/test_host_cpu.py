"""CPU tests of the product's host side (no GPU needed):

  - the C-ABI library loads and exports every symbol include/tbf.h declares;
  - a host-only engine (device = -1) builds the same tonegen template as the oracle
    (wave bank, envelopes, key-compression table, play matrix), bit for bit;
  - its control plane emits, block by block, the same core programs as the oracle's
    oscGenerateFragment restatement (src/tonegen.cpp:3218-3566) under an event script;
  - the render entry points refuse to run without a device (no CPU fallback);
  - the instance sharding used by bench.py --gpus N covers every instance exactly once
    (world_size-2 gloo run, one engine per rank).
"""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

import scenarios as S
from orc_bind import Template

ROOT = Path(__file__).resolve().parents[1]
T = pytest.importorskip("tunebfree_amd")


def _header_symbols():
    src = (ROOT / "include" / "tbf.h").read_text()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tbf_[a-z0-9_]+)\s*\(", src)))


def test_abi_exports_every_declared_symbol():
    lib = T.load_library()
    names = _header_symbols()
    assert len(names) >= 18
    for n in names:
        assert hasattr(lib, n), n
    # every non-test entry point has a ctypes signature in the host mirror
    assert {n for n in names if not n.startswith("tbf_debug_")} == set(T.engine.SIGNATURES)
    assert lib.tbf_abi_version() == 1


def test_integration_lv2_binding_is_the_compiled_one():
    """INTEGRATION.md section 2's synthSound patch is the marked section of
    tunebfree_amd/hosts/lv2_synth.h, which libtbf_lv2.so compiles (b_synth/lv2.cpp:212's
    uint32_t synthSound (B3S*, uint32_t written, uint32_t nframes, float**))."""
    h = (ROOT / "tunebfree_amd" / "hosts" / "lv2_synth.h").read_text()
    blk = h.split("/* --8<-- INTEGRATION.md section 2 */\n", 1)[1].split("/* -->8-- */", 1)[0].rstrip()
    doc = (ROOT / "INTEGRATION.md").read_text()
    sec = doc.split("## 2.", 1)[1].split("## 3.", 1)[0]
    code = sec.split("```c++\n", 1)[1].split("```", 1)[0]
    assert code == '#include "tbf.h"\n\n' + blk + "\n"
    assert "static uint32_t synthSound (B3S* b3s, uint32_t written, uint32_t nframes, float** out)" in blk
    lv2 = C.CDLL(str(ROOT / "tunebfree_amd" / "libtbf_lv2.so"))
    for n in ("tbf_lv2_synth_sound", "tbf_lv2_key", "tbf_lv2_instantiate"):
        assert hasattr(lv2, n), n


def _bind_debug(lib):
    lib.tbf_debug_contrib.restype = C.c_int
    lib.tbf_debug_contrib.argtypes = [C.c_void_p, C.c_uint32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_uint32]
    lib.tbf_debug_tables.restype = C.c_int
    lib.tbf_debug_tables.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.tbf_debug_step.restype = C.c_int
    lib.tbf_debug_step.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]
    lib.tbf_debug_render_program.restype = C.c_int
    lib.tbf_debug_render_program.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]


def _orc_bind_debug(lib):
    lib.orc_template_contrib.restype = C.c_int
    lib.orc_template_contrib.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    lib.orc_debug_program.restype = C.c_int
    lib.orc_debug_program.argtypes = [C.c_void_p, C.c_void_p, C.c_int]


@pytest.mark.parametrize("sr,seed,tuning", [(48000.0, 7, None), (44100.0, 3, "19TET"), (96000.0, 11, "p4")])
def test_host_template_matches_oracle(oracle, sr, seed, tuning):
    import json
    mts = None
    if tuning:
        mts = np.array(json.loads((ROOT / "tests" / "golden" / "tunings.json").read_text())[tuning], np.float64)
    ot = Template(oracle, sr=sr, mts128=mts, seed=seed)
    eng = T.Engine(sample_rate=sr, device=-1)
    tid = eng.template(mts128=mts, seed=seed)
    ob, ol = ot.bank()
    pb, pl = eng.template_bank(tid)
    assert np.array_equal(ol, pl)
    assert np.array_equal(ob.view(np.uint32), pb.view(np.uint32))
    lib = T.load_library()
    _bind_debug(lib)
    _orc_bind_debug(oracle)
    a, r, k = (np.zeros((9, 128), np.float32), np.zeros((9, 128), np.float32), np.zeros(128, np.float32))
    assert lib.tbf_debug_tables(eng._h, tid, a.ctypes.data, r.ctypes.data, k.ctypes.data) >= 0
    oa, orr, ok = ot.envs()
    for x, y in ((a, oa), (r, orr), (k, ok)):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))
    cap = 4096
    for key in list(range(0, 61)) + list(range(64, 125)) + list(range(128, 160)):
        w1, b1, l1 = np.zeros(cap, np.int16), np.zeros(cap, np.int16), np.zeros(cap, np.float32)
        w2, b2, l2 = np.zeros(cap, np.int16), np.zeros(cap, np.int16), np.zeros(cap, np.float32)
        n1 = lib.tbf_debug_contrib(eng._h, tid, key, w1.ctypes.data, b1.ctypes.data, l1.ctypes.data, cap)
        n2 = oracle.orc_template_contrib(ot.ptr, key, w2.ctypes.data, b2.ctypes.data, l2.ctypes.data, cap)
        assert n1 == n2, key
        assert np.array_equal(w1[:n1], w2[:n1]) and np.array_equal(b1[:n1], b2[:n1]), key
        assert np.array_equal(l1[:n1].view(np.uint32), l2[:n1].view(np.uint32)), key
    eng.close()


def _oracle_program(oracle, inst_ptr):
    buf = np.zeros(9 * 1100, np.float32)
    n = oracle.orc_debug_program(inst_ptr, buf.ctypes.data, 1100)
    e = buf[: 9 * n].reshape(n, 9)
    out, prev = [], None
    for row in e:  # fold the wrap-split second halves (same wheel, consecutive)
        w = int(row[0])
        if prev is not None and w == prev:
            continue
        prev = w
        er = int(row[2])
        env, r = (0, 0) if er < 0 else ((1, er) if er < 8 else (2, er - 8))
        out.append((w, env, r, row[3:9].copy()))
    return out


def _engine_program(lib, eng, i, lazy=False):
    buf = np.zeros(9 * 600, np.float32)
    fn = lib.tbf_debug_render_program if lazy else lib.tbf_debug_step
    n = fn(eng._h, i, buf.ctypes.data, 600)
    assert n >= 0
    return buf[: 9 * n].reshape(n, 9)


def _events_by_block(scen):
    by = {}
    for (b, kind, a, v) in scen:
        by.setdefault(b, []).append((kind, a, v))
    return by


@pytest.mark.parametrize("lazy", [False, True])
@pytest.mark.parametrize("scen", ["events", "sweep", "reroute", "retune"])
def test_control_plane_programs_match_oracle(oracle, lazy, scen, tunings):
    """Block-by-block core programs of the host control plane vs the oracle's
    oscGenerateFragment (active list order, wheel, envelope row, all six gains).
    lazy=False steps the tonegen control every block (tbf_debug_step); lazy=True makes
    exactly the step a render makes per block (tbf_debug_render_program: only when
    something changed), so a change the render path fails to pick up shows here."""
    from orc_bind import Chain
    _orc_bind_debug(oracle)
    lib = T.load_library()
    _bind_debug(lib)
    tpl = Template(oracle, seed=7)
    eng = T.Engine(device=-1)
    tid = eng.template(seed=7)
    # retune: the instances switch to a 19-TET template and back (tbf_instance_retune)
    m19 = np.array(tunings["19TET"], np.float64)
    tpls, tids = [tpl, Template(oracle, mts128=m19, seed=8)], [tid, eng.template(mts128=m19, seed=8)]
    n_inst, nblocks = 3, 64
    seeds = [1000 + i for i in range(n_inst)]
    eng.add_instances([tid] * n_inst, seeds)
    chains = [Chain(oracle, tpl, s) for s in seeds]
    fn = {"events": S.event_scenario, "sweep": S.sweep_scenario, "reroute": S.reroute_scenario,
          "retune": lambda i: S.retune_scenario(i, at=20, to=1) + [(44, "retune", 0, 0), (44, "note", 62, 1)]}[scen]
    scens = [_events_by_block(fn(i)) for i in range(n_inst)]
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
            op = _oracle_program(oracle, chains[i].ptr)
            pp = _engine_program(lib, eng, i, lazy)
            assert len(op) == len(pp), (blk, i)
            for (w, env, r, g), q in zip(op, pp):
                assert (w, env) == (int(q[0]), int(q[1])), (blk, i)
                if env:
                    assert r == int(q[2]), (blk, i)
                    assert np.array_equal(g.view(np.uint32), q[3:9].view(np.uint32)), (blk, i, w)
                else:
                    assert np.array_equal(g[:3].view(np.uint32), q[3:6].view(np.uint32)), (blk, i, w)
                checked += 1
    assert checked > 1000
    eng.close()


def test_render_refuses_without_device():
    """The product has no CPU path: a host-only engine refuses to render."""
    eng = T.Engine(device=-1)
    tid = eng.template(seed=1)
    eng.add_instances([tid], [1])
    with pytest.raises(T.TbfError):
        eng.render(1)
    with pytest.raises(T.TbfError):
        eng.synth_sound(64)
    eng.close()


def test_param_and_note_validation():
    eng = T.Engine(device=-1)
    tid = eng.template(seed=1)
    eng.add_instances([tid, tid], [1, 2])
    with pytest.raises(T.TbfError):
        eng.note(5, 60, 1)           # no such instance
    with pytest.raises(T.TbfError):
        eng.set_param(0, 9999, 1.0)  # unknown parameter id
    with pytest.raises(T.TbfError):
        eng.add_instances([77], [1])  # unknown template
    eng.note(0, 60, 1)
    eng.set_param(1, S.P_DRAWBAR + 2, 4)
    assert eng.n_instances == 2
    eng.close()


# ---------------------------------------------------------------- N>1 sharding (gloo)
def _digest(lib, eng, n, steps):
    import hashlib
    out = []
    for i in range(n):
        h = hashlib.sha256()
        for _ in range(steps):
            h.update(_engine_program(lib, eng, i).tobytes())
        out.append(h.hexdigest())
    return out


def _rank_main(rank, world, port, n_total, q):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tunebfree_amd.shard import shard
    lib = T.load_library()
    _bind_debug(lib)
    first, cnt = shard(n_total, rank, world)
    eng = T.Engine(device=-1)
    tid = eng.template(seed=7)
    eng.add_instances([tid] * cnt, [1000 + first + i for i in range(cnt)])
    for i in range(cnt):
        for (_, kind, a, v) in S.bench_scenario(first + i):
            (eng.note if kind == "note" else eng.set_param)(i, a, v)
    dig = _digest(lib, eng, cnt, 3)
    got = [None] * world
    dist.all_gather_object(got, (first, cnt, dig))
    if rank == 0:
        q.put(got)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_world2_gloo():
    import multiprocessing as mp
    import socket
    from tunebfree_amd.shard import shard
    n_total = 7
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank_main, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=240)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    covered = sorted(i for (f, c, _) in got for i in range(f, f + c))
    assert covered == list(range(n_total))
    # each rank's instances are exactly the single-process engine's instances
    lib = T.load_library()
    _bind_debug(lib)
    eng = T.Engine(device=-1)
    tid = eng.template(seed=7)
    eng.add_instances([tid] * n_total, [1000 + i for i in range(n_total)])
    for i in range(n_total):
        for (_, kind, a, v) in S.bench_scenario(i):
            (eng.note if kind == "note" else eng.set_param)(i, a, v)
    ref = _digest(lib, eng, n_total, 3)
    merged = [d for (f, c, dig) in sorted(got) for d in dig]
    assert merged == ref
    assert shard(8 * 4096, 3, 8) == (3 * 4096, 4096)


# ---------------------------------------------------------------- exact shortcuts
def _exact(op, rows):
    lib = T.load_library()
    lib.tbf_debug_exact.restype = C.c_int
    lib.tbf_debug_exact.argtypes = [C.c_int32, C.c_void_p, C.c_void_p, C.c_uint32]
    a = np.ascontiguousarray(rows, np.float64).reshape(-1, 3)
    out = np.zeros((len(a), 2), np.float64)
    assert lib.tbf_debug_exact(op, a.ctypes.data, out.ctypes.data, len(a)) == 0
    return out


def test_phase_closed_form_is_exact():
    """csrc/tbf_exact.h phase_run: when it accepts a run, v0 + j*D equals the reference's
    repeated `vib += depth * vibSpeed` (src/reverb.cpp:479-496) for every j <= m."""
    rng = np.random.default_rng(5)
    depth = np.array([0.003251, 0.002999, 0.002917, 0.002749, 0.002503, 0.002423, 0.002146, 0.002088])
    ds = list(depth * 0.06) + list(depth * 1.06) + list(rng.uniform(1e-7, 0.5, 40))
    v0s = list(rng.integers(-2 ** 31, 2 ** 31, 200).astype(np.float64) - 1073741823.0)
    for k in range(-20, 32):  # values hugging binade edges, both signs
        for eps in (0.0, 1e-16, 3e-16, 1e-12, 1e-6, 1e-3):
            for sg in (1.0, -1.0):
                v0s += [sg * 2.0 ** k * (1 + eps), sg * 2.0 ** k * (1 - eps / 2)]
    rows = [(v, d, 64) for v in v0s for d in ds]
    out = _exact(0, rows)
    accepted = 0
    for (v0, d, m), (ok, D) in zip(rows, out):
        if not ok:
            continue
        accepted += 1
        v = np.float64(v0)
        for j in range(1, int(m) + 1):
            v = v + np.float64(d)
            assert v == np.float64(v0) + np.float64(j) * np.float64(D), (v0, d, j)
    # the kernel's fast path covers the reference's own phases (rand() - RAND_MAX/2 seeds)
    real = [(v, d, 64) for v in v0s[:200] for d in ds[:16]]
    assert _exact(0, real)[:, 0].mean() > 0.99
    assert 0.1 * len(rows) < accepted < len(rows)  # both outcomes exercised


def test_count_and_wrap_shortcuts():
    rows, want = [], []
    for d in (560, 756, 1007, 3):
        for c0 in (-1, 0, 1, d - 64, d - 1, d, d + 1, d + 50):
            for n in (0, 1, 63, 64, 65, 128):
                c = c0
                for _ in range(n):  # src/reverb.cpp: count++; if (count < 0 || count > d) count = 0
                    c += 1
                    if c < 0 or c > d:
                        c = 0
                rows.append((c0, d, n))
                want.append(c)
    assert [int(x) for x in _exact(1, rows)[:, 0]] == want
    xs = np.array([0.0, 0.25, 0.999999999, 1.0, 1.5, 1.9999999, 2.0, 2.5, -0.25, 7.75, np.nan, np.inf])
    got = _exact(2, [(x, 0, 0) for x in xs])[:, 0]
    ref = np.fmod(xs, 1.0)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    assert np.array_equal(got[~np.isnan(ref)], ref[~np.isnan(ref)])


def test_dither_jump_table_matches_literal_xorshift():
    """The kernels generate the Airwindows xorshift32 dither streams (src/overdrive.cpp:
    158-160, src/reverb.cpp:775-783) by GF(2) jumps instead of 64-128 serial steps; the
    jump equals the literal recurrence for every k the kernels use (0..128).  The host
    hook evaluates it as the kernels do, from the nibble-sliced table (8 entries per state),
    and fails if that ever differs from the 32 bit-row form."""
    rng = np.random.default_rng(5)
    seeds = [1, 16386, 0xFFFFFFFF, 0x80000000, 12345] + [int(x) for x in rng.integers(1, 2 ** 32, 40)]
    rows = [(x0, k, 0) for x0 in seeds for k in (0, 1, 2, 63, 64, 65, 127, 128)]
    out = _exact(3, rows)
    assert np.array_equal(out[:, 0], out[:, 1])
    x, seq = 16386, []
    for _ in range(5):  # spot check of the literal stream itself
        x ^= (x << 13) & 0xFFFFFFFF
        x ^= x >> 17
        x ^= (x << 5) & 0xFFFFFFFF
        seq.append(x)
    assert [int(v) for v in _exact(3, [(16386, k, 0) for k in range(1, 6)])[:, 1]] == seq


def test_phase_cache_matches_phase_run():
    """The reverb core caches each line's closed-form phase step per binade
    (phase_run_cached); along long runs it decides exactly like phase_run."""
    rng = np.random.default_rng(11)
    v0s = [float(x) - 2147483647 // 2 for x in rng.integers(0, 2 ** 31 - 1, 12)] + [3.0, -3.0, 1e-3, 0.75]
    ds = [0.003251 * 0.06, 0.002088 * 0.06, 0.0, 1.0 / 3.0]
    out = _exact(4, [(v, d, 64) for v in v0s for d in ds])
    assert out[:, 0].sum() == 0
    assert out[:, 1].sum() > 0.9 * 4096 * len(v0s) * 2  # the cache serves almost every sub-block


def test_glibc_rand_jump_matches_literal_draws():
    """csrc/tbf_rand.h: GlibcRand::discard (k) -- the polynomial jump x^k mod
    (x^31 - x^28 - 1) over Z/2^32 that the device template builder uses per chunk --
    leaves the same stream as k literal rand() calls (src/tonegen.cpp:1449 draws)."""
    rows = [(s, k, 0) for s in (1, 7, 12345) for k in (0, 1, 2, 30, 31, 32, 61, 310, 4097, 359853)]
    out = _exact(5, rows)
    assert np.array_equal(out[:, 0], out[:, 1])


def test_config_api_semantics():
    """tbf_config_set / tbf_config_parse return codes (include/tbf.h): applied, ignored
    (keys of other modules, and keys the reference stores but never reads on this path),
    bad values (getConfigParameter_*'s ranges, src/cfgParser.cpp:453-620, and malformed
    list keys: nothing assigned), engine-wide keys after instances exist, and the
    parser's line-numbered errors."""
    import scenarios as S
    eng = T.Engine(device=-1)
    assert eng.config_set("whirl.horn.radius", 25) == 0
    assert eng.config_set("WHIRL.DRUM.RADIUS", 18) == 0  # strcasecmp, as the reference
    assert eng.config_set("midi.upper.channel", 1) == 1
    assert eng.config_set("overdrive.character", 0.5) == 1
    assert eng.config_set("xov.ctl_biased", 0.3) == 1
    for k, v in (("scanner.hz", 3.9), ("whirl.drum.filter.type", 9), ("reverb.mix", 1.5),
                 ("whirl.horn.brakepos", -0.1), ("osc.perc.bus.trig", -2)):
        with pytest.raises(T.TbfError, match="-22"):
            eng.config_set(k, v)
    # keys the reference stores but never reads on this path
    for k, v in (("osc.tuning", 440), ("osc.temperament", "gear60"), ("osc.eqv.5", 0.5),
                 ("whirl.horn.comb.a.feedback", -0.5)):
        assert eng.config_set(k, v) == 1
    # the tone generator's list keys: well formed, or refused whole
    assert eng.config_set("osc.crosstalk.k60", "1:45:0.02, 4:57:0.01") == 0
    assert eng.config_set("osc.taper.k60.b2.t57", 0.8) == 0
    assert eng.config_set("osc.harmonic.w40.f3", 0.1) == 0
    assert eng.config_set("osc.eq.macro", "peak24") == 0
    for k, v in (("osc.crosstalk.k60", "1:45:0.02,4:57"), ("osc.crosstalk.k0", "1:45:0.02"),
                 ("osc.taper.k60.b0.t57", 0.5), ("osc.taper.k60.b2.t257", 0.5), ("osc.harmonic.0", 0.1),
                 ("osc.harmonic.w0.f2", 0.1), ("osc.terminal.t3.w300", 0.1), ("osc.eq.macro", "flat"),
                 ("osc.transformer-crosstalk", 0.02)):
        with pytest.raises(T.TbfError, match="-22"):
            eng.config_set(k, v)
    assert eng.config_set("osc.transformer-crosstalk", 0) == 0
    # the compact whirl ring window follows the geometry (512 / 1024 / 2048) ...
    e2 = T.Engine(device=-1)
    assert e2.layout()["wring_len"] == 512
    e2.config_set("whirl.horn.radius", 60)
    assert e2.layout()["wring_len"] == 1024
    e2.close()
    e2 = T.Engine(sample_rate=96000.0, device=-1)
    assert e2.layout()["wring_len"] == 1024
    e2.config_set("whirl.horn.radius", 80)
    assert e2.layout()["wring_len"] == 2048
    e2.close()
    # ... and geometry beyond the reference's 2048-sample ring is refused, leaving the
    # engine as it was
    with pytest.raises(T.TbfError, match="-22"):
        eng.config_set("whirl.horn.radius", 1000)
    assert eng.config_set("whirl.horn.radius", 25) == 0
    txt = "# a cfg file\n\n  scanner.hz = 6.5  # comment\nmidi.lower.channel=2\nreverb.mix=0.3\n"
    assert eng.config_parse(txt) == 2
    with pytest.raises(T.TbfError, match="line 2"):
        eng.config_parse("reverb.mix=0.2\nnot a key value line\n")
    with pytest.raises(T.TbfError, match="line 3"):
        eng.config_parse("reverb.mix=0.2\n\nscanner.hz=30\n")
    # all or nothing: a bad line leaves even the earlier, well-formed keys unapplied
    w0 = eng.layout()["wring_len"]
    with pytest.raises(T.TbfError, match="line 2"):
        eng.config_parse("whirl.horn.radius = 80\nnot a key value line\n")
    assert eng.layout()["wring_len"] == w0
    assert eng.config_parse("whirl.horn.radius = 80\n") == 1 and eng.layout()["wring_len"] > w0
    assert eng.config_parse("whirl.horn.radius = 25\n") == 1 and eng.layout()["wring_len"] == w0
    tid = eng.template(seed=3)
    eng.add_instances([tid], [5])
    # engine-wide tables are fixed once instances exist; per-instance / template keys are not
    for k, v in (("whirl.horn.radius", 20), ("scanner.modulation.v1", 4), ("whirl.horn.filter.a.hz", 3000)):
        with pytest.raises(T.TbfError, match="-16"):
            eng.config_set(k, v)
    assert eng.config_set("reverb.mix", 0.2) == 0
    assert eng.config_set("osc.attack.model", "cosine") == 0
    assert eng.config_set("whirl.speed-preset", 2) == 0
    eng.close()
    assert S.CFG_SETS  # the parity sets: test_oracle_cpu / test_gpu_parity


def test_device_templates_refused_on_host_engine():
    eng = T.Engine(sample_rate=48000.0, device=-1)
    with pytest.raises(RuntimeError):
        eng.templates([7])
    eng.close()


def test_host_templates_vs_reference_pins(tunings):
    """The product's host template builder (tbf_template_create on a host-only engine)
    gives the wave banks, lengths, envelopes, key-compression tables and play matrices of
    the reference's own src/tonegen.cpp builders (digests in tests/golden/template_pins.json,
    see tests/golden/make_template_pins.py), bit for bit: 7 tunings x 48 / 96 kHz and the
    osc.* cfg sets (envelope models, wheel EQ, harmonics, terminal / taper / crosstalk
    lists, crosstalk levels, contribution floor / minimum)."""
    import hashlib
    import json
    from orc_bind import contrib_from
    pins = json.loads((ROOT / "tests" / "golden" / "template_pins.json").read_text())
    lib = T.load_library()
    _bind_debug(lib)
    engines = {}
    for p in pins:
        key = (p["sr"], p.get("cfg"))
        if key not in engines:
            engines[key] = T.Engine(sample_rate=p["sr"], device=-1)
            if p.get("cfg"):
                engines[key].config(S.CFG_SETS[p["cfg"]])
        eng = engines[key]
        m = None if tunings[p["tuning"]] is None else np.array(tunings[p["tuning"]], np.float64)
        tid = eng.template(mts128=m, seed=p["seed"])
        bank, lens = eng.template_bank(tid)
        a, r, k = np.zeros((9, 128), np.float32), np.zeros((9, 128), np.float32), np.zeros(128, np.float32)
        assert lib.tbf_debug_tables(eng._h, tid, a.ctypes.data, r.ctypes.data, k.ctypes.data) == 0
        got = {"bank": bank, "lens": lens, "attack": a, "release": r, "keycomp": k,
               "contrib": contrib_from(lambda kk, w, b, lv, cap: lib.tbf_debug_contrib(eng._h, tid, kk, w, b, lv, cap))}
        for key, v in got.items():
            assert hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest() == p[key], \
                (p["tuning"], p["sr"], p.get("cfg"), key)
    for e in engines.values():
        e.close()


def _bench_json(args, nproc=None, port=None):
    import json
    import subprocess
    import sys
    cmd = [sys.executable]
    if nproc:
        cmd += ["-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}", "--master-addr",
                "127.0.0.1", f"--master-port={port}"]
    cmd += [str(ROOT / "bench.py")] + args
    out = subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=240, cwd=str(ROOT)).stdout
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out  # rank 0 alone prints, exactly one JSON line
    return json.loads(lines[0])


def test_bench_world2_dry_run_gloo():
    """bench.py itself at world size 2 (torch.distributed.run, gloo, host-only engines,
    --dry-run): the ranks take their instance ranges from tunebfree_amd.shard, run the
    timed region between barriers, reduce over ranks, and rank 0 prints one JSON line
    with the contract's keys.  The sum over ranks of per-instance control checksums
    equals the single-process run over the whole batch, so the shards cover every
    instance exactly once with the right global indices."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    common = ["--dry-run", "1", "--steps", "2", "--warmup", "1", "--check", "0"]
    one = _bench_json(common + ["--batch", "10"])
    two = _bench_json(common + ["--gpus", "2", "--batch", "5"], nproc=2, port=port)
    for d, n in ((one, 1), (two, 2)):
        for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                  "scaling", "vs_baseline", "dtype", "data", "config"):
            assert k in d, k
        assert d["n_gpus"] == n and d["scaling"] == "weak" and d["value"] > 0
    assert two["dry_run"]["shard_rank0"] == [0, 5]
    assert two["dry_run"]["checksum"] == one["dry_run"]["checksum"]
    # the driver's command form: `bench.py --gpus 2` with no launcher starts the two ranks itself
    self_launched = _bench_json(common + ["--gpus", "2", "--batch", "5"])
    assert self_launched["n_gpus"] == 2
    assert self_launched["dry_run"]["shard_rank0"] == [0, 5]
    assert self_launched["dry_run"]["checksum"] == one["dry_run"]["checksum"]


def test_bench_world_size_mismatch_fails():
    """A launcher world size that differs from --gpus is an error (exit 2), not a silent
    one-GPU run reported as N."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dry-run", "1"],
                         env=env, capture_output=True, text=True, timeout=120, cwd=str(ROOT))
    assert out.returncode == 2, out.stderr[-2000:]
    assert "WORLD_SIZE=1" in out.stderr and not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]


def test_drawbar_setting_out_of_range_ignored():
    """setDrawBar asserts 0 <= setting < 9 (src/tonegen.cpp:2741); the engine ignores a
    setting outside that (no drawbar change, no gain change), on the host front end and in
    the device front end's packing (frontParam: setting 15 = ignored)."""
    lib = T.load_library()
    _bind_debug(lib)
    eng = T.Engine(device=-1)
    tid = eng.template(seed=7)
    eng.add_instances([tid], [3])
    for k in S.chord_for(0):
        eng.note(0, k, 1)
    before = [_engine_program(lib, eng, 0, False) for _ in range(3)][-1]
    for bad in (9, 12):
        eng.set_param(0, S.P_DRAWBAR + 2, bad)
        eng.set_param(0, S.P_BUS_DRAWBAR + 11, bad)
    after = [_engine_program(lib, eng, 0, False) for _ in range(3)][-1]
    assert np.array_equal(before.view(np.uint32), after.view(np.uint32))
    eng.set_param(0, S.P_DRAWBAR + 2, 3)
    moved = [_engine_program(lib, eng, 0, False) for _ in range(3)][-1]
    assert not np.array_equal(before.view(np.uint32), moved.view(np.uint32))
    eng.close()


def test_host_pool_runs_every_task_once():
    """The host worker pool (HostPool, csrc/tbf_engine.cpp) behind the control plane's
    parallel sections: a job ends when its tasks are done, and a worker woken late must
    find that job's tasks taken rather than run a later job's twice.  20000 jobs of 1..40
    tasks back to back, every task counted (tbf_debug_pool_check), with the pool at 16
    threads."""
    import os
    import subprocess
    import sys
    code = ("import ctypes as C, tunebfree_amd as T; lib = T.load_library(); "
            "lib.tbf_debug_pool_check.restype = C.c_int; lib.tbf_debug_pool_check.argtypes = [C.c_uint32]; "
            "print(lib.tbf_debug_pool_check(20000))")
    env = dict(os.environ, TBF_HOST_THREADS="16")
    out = subprocess.run([sys.executable, "-c", code], env=env, cwd=str(ROOT), capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.strip().splitlines()[-1] == "0"

