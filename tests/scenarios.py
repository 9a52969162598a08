"""Event scripts shared by the oracle, reference-checker and GPU parity tests.

A scenario is a list of (block, kind, a, b) events applied before rendering
`block`: kind "note" (a=key, b=on) or "param" (a=param id, b=value).  Param ids
are the CLAP ids of src/clap.cpp:31-48 plus the extension ids of oracle/orc.h.
"""
from __future__ import annotations

# CLAP parameter ids (src/clap.cpp:31-48)
P_DRAWBAR = 0
P_VIBRATO, P_VIBRATO_TYPE, P_DRUM, P_HORN = 9, 10, 11, 12
P_OVERDRIVE, P_CHARACTER, P_REVERB = 13, 14, 15
P_PERC, P_PERC_VOL, P_PERC_DECAY, P_PERC_HARM = 16, 17, 18, 19
P_BUS_DRAWBAR, P_VIB_LOWER, P_SWELL, P_WHIRL_BYPASS = 100, 130, 131, 132


def jazz1_params(character=0.5, reverb=0.1):
    """pgm/default.pgm:27-36 "Jazz 1 all" via the CLAP parameter surface:
    drawbars 888 0000 000, perc on/soft/fast/3rd, vibrato C3 upper, overdrive on,
    rotary chorale (horn+drum slow = rev option 4)."""
    ev = []
    for i, v in enumerate([8, 8, 8, 0, 0, 0, 0, 0, 0]):
        ev.append(("param", P_DRAWBAR + i, v))
    ev += [
        ("param", P_PERC, 1), ("param", P_PERC_VOL, 0), ("param", P_PERC_DECAY, 1),
        ("param", P_PERC_HARM, 0), ("param", P_VIBRATO_TYPE, 5), ("param", P_VIBRATO, 1),
        ("param", P_OVERDRIVE, 1), ("param", P_CHARACTER, character), ("param", P_REVERB, reverb),
        ("param", P_DRUM, 1), ("param", P_HORN, 1),
    ]
    return ev


def chord_for(i):
    root = 48 + (i % 24)
    return [root, root + 4, root + 7, root + 12]


def bench_scenario(i, full=True):
    """BASELINE configs 2/3: instance i plays chord root 48+(i mod 24) + {0,4,7,12}."""
    ev = [(0, k, a, b) for (k, a, b) in (jazz1_params() if full else
          [("param", P_DRAWBAR + j, v) for j, v in enumerate([8, 8, 8, 0, 0, 0, 0, 0, 0])]
          + [("param", P_VIBRATO_TYPE, 5), ("param", P_VIBRATO, 1)])]
    ev += [(0, "note", k, 1) for k in chord_for(i)]
    return ev


def event_scenario(i):
    """SURVEY.md s8(c) golden plan: chord at block 0, chord change + drawbar change +
    rotary fast->slow at block 32, note-off at block 48 (release + wheel removal)."""
    ev = bench_scenario(i)
    ev += [(0, "param", P_DRUM, 2), (0, "param", P_HORN, 2)]  # start fast
    c0 = chord_for(i)
    c1 = chord_for(i + 5)
    ev += [(32, "note", k, 0) for k in c0[:2]]
    ev += [(32, "note", k, 1) for k in c1[:3]]
    ev += [(32, "param", P_DRAWBAR + 3, 6), (32, "param", P_DRUM, 1), (32, "param", P_HORN, 1)]
    ev += [(40, "param", P_PERC, 0), (40, "param", P_VIB_LOWER, 1), (40, "note", 128 + 36 + (i % 12), 1)]
    ev += [(48, "note", k, 0) for k in set(c0[2:] + c1[:3])]
    ev += [(56, "param", P_VIBRATO_TYPE, 2), (56, "note", 60 + (i % 7), 1), (56, "param", P_SWELL, 0.5)]
    return ev


class GlibcRand:
    """glibc srand()/rand() (TYPE_3 additive generator), for event scripts that follow
    the reference's rand()-driven control code."""

    def __init__(self, seed):
        seed = seed or 1
        r = [0] * 34
        r[0] = seed & 0x7FFFFFFF if seed < 2 ** 31 else seed - 2 ** 32
        for i in range(1, 31):
            hi, lo = divmod(r[i - 1], 127773) if r[i - 1] >= 0 else (-((-r[i - 1]) // 127773), -((-r[i - 1]) % 127773))
            w = 16807 * lo - 2836 * hi
            r[i] = w + 2147483647 if w < 0 else w
        for i in range(31, 34):
            r[i] = r[i - 31]
        self.r = [x & 0xFFFFFFFF for x in r]
        for _ in range(310):
            self._step()

    def _step(self):
        v = (self.r[-31] + self.r[-3]) & 0xFFFFFFFF
        self.r.append(v)
        del self.r[0]
        return v >> 1

    def next(self):
        return self._step()


SWEEP_CHARACTER = (0.0, 0.3, 0.9, 1.0)
SWEEP_REVERB = (0.0, 0.7, 1.0)


def sweep_scenario(i):
    """Parameter regions beyond the bench registration ("what's weak" 2),
    varied with the instance index i:
      - overdrive character SWEEP_CHARACTER[i % 4] (fsetCharacter, src/overdrive.cpp:552-574:
        0 iterations / density 0 takes the 1 - cos branch, 1.0 squares to 16 sin passes);
        instance i % 7 == 6 runs clean
      - reverb mix SWEEP_REVERB[i % 3] (setReverbMix, src/reverb.cpp:233: 1.0 drops the dry path)
      - percussion volume/decay/harmonic = bits 0/1/2 of i (normal/soft, fast/slow, 2nd/3rd),
        retriggered after all upper keys go up (src/tonegen.cpp:3257-3327)
      - i % 3 == 0: a 13-key upper cluster (key-compression table past index 12),
        otherwise a 4-note chord
      - pedal drawbars 8 0 6 0 ... and pedal keys 256..383 (src/midi.cpp:1469-1484)
      - rotary: even i starts stopped (rev option 0, free stop), goes fast at block 12,
        stops again at block 36 (deceleration to 0), chorale at 60; odd i the reverse
        order from fast."""
    ev = [(0, k, a, b) for (k, a, b) in jazz1_params(character=SWEEP_CHARACTER[i % 4],
                                                       reverb=SWEEP_REVERB[i % 3])]
    if i % 7 == 6:
        ev.append((0, "param", P_OVERDRIVE, 0))
    ev += [(0, "param", P_PERC_VOL, (i >> 0) & 1), (0, "param", P_PERC_DECAY, 1 - ((i >> 1) & 1)),
           (0, "param", P_PERC_HARM, (i >> 2) & 1)]
    for j, v in enumerate((8, 0, 6, 0, 0, 0, 0, 0, 4)):
        ev.append((0, "param", P_BUS_DRAWBAR + 18 + j, v))
    keys = list(range(48 + i % 5, 61 + i % 5)) if i % 3 == 0 else chord_for(i)
    ev += [(0, "note", k, 1) for k in keys]
    ped = 256 + 24 + (i % 12)
    ev += [(0, "note", ped, 1), (20, "note", ped, 0), (21, "note", ped + 5, 1), (44, "note", ped + 5, 0),
           (45, "note", 383, 1), (46, "note", 256, 1)]
    # all upper keys up, then a retrigger (percussion fires on the first key down again)
    ev += [(24, "note", k, 0) for k in keys]
    ev += [(28, "note", k, 1) for k in keys[:3]]
    ev += [(50, "note", 40 + (i % 9), 1), (52, "note", 127, 1)]
    rot = [(0, 0, 0), (12, 2, 2), (36, 0, 0), (60, 1, 1)] if i % 2 == 0 else \
          [(0, 2, 2), (12, 0, 0), (30, 2, 2), (60, 0, 0)]
    for (b, d, h) in rot:
        ev += [(b, "param", P_DRUM, d), (b, "param", P_HORN, h)]
    return ev


def reroute_scenario(i):
    """Drawbar, routing and percussion changes with no key event in the same block
    (drawbar sweeps, vibrato switches): the active wheels keep envelope-free entries
    but their routed sums change, which the reference applies from the next block
    (src/tonegen.cpp:3427-3485)."""
    return bench_scenario(i) + [(0, "note", 128 + 40, 1), (19, "param", P_DRAWBAR + 4, 7),
                                (23, "param", P_VIBRATO, 0), (26, "param", P_VIB_LOWER, 1),
                                (29, "param", P_BUS_DRAWBAR + 11, 3), (33, "param", P_PERC, 0),
                                (37, "param", P_PERC, 1), (41, "param", P_PERC_HARM, 1),
                                (44, "param", P_DRAWBAR + 0, 0), (45, "param", P_DRAWBAR + 1, 2)]


# cfg key sets (tbf_config_set / the oracle's orc_cfg / the reference structs' fields):
# each reshapes the tables the engine builds after it (cfg keys)
CFG_SETS = {
    "geometry": {"whirl.horn.radius": 25, "whirl.drum.radius": 18, "whirl.mic.distance": 60,
                 "whirl.horn.offset.x": 3, "whirl.horn.offset.z": -2},
    # a wider horn: the compact whirl ring window doubles to 1024 at 48 kHz (2048 at 96)
    "geometry_wide": {"whirl.horn.radius": 60, "whirl.drum.radius": 30, "whirl.mic.distance": 50},
    "filters": {"whirl.drum.filter.type": 6, "whirl.drum.filter.hz": 700, "whirl.drum.filter.q": 1.2,
                "whirl.drum.filter.gain": -20, "whirl.horn.filter.a.hz": 3800, "whirl.horn.filter.a.q": 1.8,
                "whirl.horn.filter.b.type": 7, "whirl.horn.filter.b.hz": 350, "whirl.horn.filter.b.gain": -25,
                "whirl.horn.filter.b.q": 1.3},
    "brake": {"whirl.speed-preset": 1, "whirl.horn.brakepos": 0.75, "whirl.drum.brakepos": 0.5,
              "whirl.horn.slowrpm": 48, "whirl.horn.fastrpm": 400, "whirl.drum.slowrpm": 40,
              "whirl.drum.fastrpm": 342, "whirl.horn.acceleration": 0.3, "whirl.drum.deceleration": 2.0},
    "mix": {"whirl.horn.level": 0.8, "whirl.horn.leak": 0.1, "whirl.horn.mic.angle": 150,
            "whirl.horn.width": 0.4, "whirl.drum.width": -0.3, "scanner.hz": 6.5, "scanner.modulation.v3": 7.5,
            "scanner.modulation.v1": 2.0, "reverb.mix": 0.3, "osc.perc.normal": 0.9, "osc.perc.soft": 0.4,
            "osc.perc.gain": 9, "osc.perc.bus.a": 2, "osc.perc.bus.b": 5, "osc.perc.bus.trig": 7},
    "envelopes": {"osc.attack.model": "shelf", "osc.release.model": "click", "osc.release.click.level": 0.4,
                  "osc.attack.click.minlength": 0.05, "osc.attack.click.maxlength": 0.4, "osc.x-precision": 0.002},
    "envelopes2": {"osc.attack.model": "cosine", "osc.release.model": "shelf", "osc.attack.click.level": 0.7,
                   "osc.attack.click.maxlength": 0.3},
    # the tone generator's list keys (oscConfig, src/tonegen.cpp:2296-2474): extra wheel
    # harmonics (all wheels / one wheel), a terminal's own mix, key tapers (a manual key
    # and a pedal), explicit key crosstalk, the spline EQ points
    "osc_lists": [("osc.harmonic.3", 0.05), ("osc.harmonic.2", 0.1), ("osc.harmonic.w40.f5", 0.2),
                  ("osc.harmonic.w40.f2", -0.05), ("osc.terminal.t57.w57", 0.9), ("osc.terminal.t57.w45", 0.05),
                  ("osc.terminal.t60.w60", 0.7), ("osc.taper.k60.b2.t57", 0.8), ("osc.taper.k60.b3.t69", 0.5),
                  ("osc.taper.k60.b8.t60", 0.3), ("osc.taper.k260.b19.t40", 1.0), ("osc.taper.k260.b20.t52", 0.6),
                  ("osc.crosstalk.k60", "1:45:0.02, 4:57:0.01,7:81:0.004"), ("osc.crosstalk.k188", "12:60:0.03"),
                  ("osc.eq.p1y", 0.8), ("osc.eq.r1y", 0.3), ("osc.eq.p4y", 0.6), ("osc.eq.r4y", -0.2)],
    # the wheel EQ macro and the default crosstalk model's levels / the contribution floor
    "osc_models": {"osc.eq.macro": "peak46", "osc.compartment-crosstalk": 0.03, "osc.transformer-crosstalk": 0,
                   "osc.terminalstrip-crosstalk": 0.005, "osc.wiring-crosstalk": 0.02,
                   "osc.contribution-floor": 0.0005, "osc.contribution-min": 0.001},
}


def cfg_scenario(i):
    """For the cfg sets: the Jazz-1 registration without its rotary selection (the cfg's
    speed preset holds at the start), chords, a note-off/on, then the rotor through
    stop -> fast -> stop (the brake positions, when set) -> slow -> stop."""
    ev = [(0, k, a, b) for (k, a, b) in jazz1_params() if a not in (P_DRUM, P_HORN)]
    ev += [(0, "param", P_PERC_VOL, i & 1), (0, "param", P_VIBRATO_TYPE, 4 + (i & 1))]
    ev += [(0, "note", k, 1) for k in chord_for(i)] + [(0, "note", 256 + 30 + i % 5, 1)]
    ev += [(20, "note", k, 0) for k in chord_for(i)] + [(22, "note", k, 1) for k in chord_for(i + 3)]
    for (b, d, h) in ((6, 0, 0), (9, 2, 2), (26, 0, 0), (48, 1, 1), (60, 0, 0)):
        ev += [(b, "param", P_DRUM, d), (b, "param", P_HORN, h)]
    return ev


WHIRL_CONTROLS = tuple(f"whirl.horn.filter.{ab}.{k}" for ab in "ab" for k in ("type", "hz", "q", "gain")) + (
    "whirl.horn.brakepos", "whirl.drum.brakepos", "whirl.horn.acceleration", "whirl.horn.deceleration",
    "whirl.drum.acceleration", "whirl.drum.deceleration")


def whirl_control_scenario(i, seed=None):
    """cfg_scenario's rotor script (stop 6, fast 9, stop 26, slow 48, stop 60) with the
    whirl's MIDI control functions (src/whirl.cpp:699-889) at seeded random values: both
    horn filters at the start, horn filter A changed on consecutive blocks (its one
    sub-block run-ahead), brake positions before the stops, ramp times before the speed
    changes, out-of-range filter settings that leave the coefficients as they were (Q at
    0, gain at +-48 dB), a brake released during the stop and a filter change while the
    whirl is bypassed."""
    import numpy as np
    g = np.random.default_rng(7000 + i if seed is None else seed)
    ev = cfg_scenario(i)

    def c(b, name, v=None):
        ev.append((b, "control", name, int(g.integers(0, 128) if v is None else v)))
    for ab in "ab":
        for k in ("type", "hz", "q", "gain"):
            c(0, f"whirl.horn.filter.{ab}.{k}")
    c(3, "whirl.horn.filter.a.hz")
    c(4, "whirl.horn.filter.a.q", 20 + int(g.integers(0, 100)))
    c(5, "whirl.horn.filter.b.gain")
    c(5, "whirl.horn.brakepos", 1 + int(g.integers(0, 127)))
    c(5, "whirl.drum.brakepos", 1 + int(g.integers(0, 127)))
    c(8, "whirl.horn.acceleration")
    c(8, "whirl.drum.acceleration")
    c(24, "whirl.horn.deceleration")
    c(24, "whirl.drum.deceleration")
    c(30, "whirl.horn.filter.a.q", 0)
    c(31, "whirl.horn.filter.b.gain", 127)
    c(32, "whirl.horn.filter.a.gain", 0)
    c(33, "whirl.horn.filter.a.type", 127)
    c(36, "whirl.horn.brakepos", 0 if i & 1 else None)
    c(40, "whirl.drum.brakepos")
    c(47, "whirl.horn.acceleration")
    c(47, "whirl.drum.deceleration")
    ev.append((50, "param", P_WHIRL_BYPASS, 1))
    c(51, "whirl.horn.filter.a.hz")
    ev.append((53, "param", P_WHIRL_BYPASS, 0))
    c(53, "whirl.horn.filter.b.hz")
    c(58, "whirl.horn.brakepos", 1 + int(g.integers(0, 127)))
    c(58, "whirl.drum.brakepos", 1 + int(g.integers(0, 127)))
    return sorted(ev, key=lambda r: r[0])


def random_drawbar_scenario(i, seed=None):
    """BASELINE config 5: upper drawbars from randomizeDrawbars (`rand() % 9` x 9,
    src/program.cpp:716-729) after srand(seed), rest of the Jazz-1 registration,
    chord root 48+(i mod 24) + {0,4,7,12}."""
    g = GlibcRand(1 + i if seed is None else seed)
    bars = [g.next() % 9 for _ in range(9)]
    ev = [(0, k, a, b) for (k, a, b) in jazz1_params()]
    ev += [(0, "param", P_DRAWBAR + j, v) for j, v in enumerate(bars)]
    ev += [(0, "note", k, 1) for k in chord_for(i)]
    return ev


def run(chain, scenario, nblocks, stages=False, templates=None):
    """Apply events at block boundaries and render; returns concatenated arrays.
    ("retune", j, 0) switches the chain to templates[j] (CLAP reinitToneGen)."""
    import numpy as np
    by_block = {}
    for (blk, kind, a, b) in scenario:
        by_block.setdefault(blk, []).append((kind, a, b))
    outs = []
    b = 0
    bounds = sorted(set([0, nblocks] + [k for k in by_block if k < nblocks]))
    for s, e in zip(bounds[:-1], bounds[1:]):
        for (kind, a, v) in by_block.get(s, []):
            if kind == "note":
                chain.note(a, v)
            elif kind == "retune":
                chain.retune(templates[a])
            elif kind == "control":
                chain.control(a, v)
            else:
                chain.param(a, v)
        outs.append(chain.render(e - s, stages=stages))
    return [np.concatenate(x) for x in zip(*outs)]


def retune_scenario(i, at=24, to=0):
    """MTS-ESP retune mid-phrase (§8(f) row 3): the Jazz-1 registration with drawbars,
    vibrato and percussion set through CLAP parameters, a chord held across the retune
    at block `at` to templates[to] (the new tone generator starts with no keys down, its
    drawbars / vibrato restored from the parameters, the routing word kept), then new
    notes on the new tuning, a vibrato-type change and a release."""
    ev = [(0, k, a, b) for (k, a, b) in jazz1_params()
          if not (i & 1 and (a <= P_DRAWBAR + 8 or a == P_HORN))]
    if i & 1:
        # drawbars never set through parameters (the instance's {8,8,6} preset plays until
        # the retune restores the parameters' defaults {7,8,8,0...}); the drum speed alone
        # (the horn parameter at its default 1: revOption 2 + 3)
        ev += [(0, "param", P_DRUM, 2)]
    else:
        ev += [(0, "param", P_DRAWBAR + 3, 5 + i % 3)]
    ev += [(0, "param", P_VIBRATO, 1), (0, "param", P_VIBRATO_TYPE, i % 6), (0, "param", P_PERC, (i >> 1) & 1)]
    ev += [(2, "note", k, 1) for k in chord_for(i)]
    ev += [(at, "retune", to, 0)]
    ev += [(at, "note", k, 1) for k in chord_for(i + 5)]
    ev += [(at + 9, "param", P_VIBRATO_TYPE, (i + 3) % 6), (at + 12, "param", P_DRAWBAR + 1, 4)]
    ev += [(at + 20, "note", k, 0) for k in chord_for(i + 5)]
    return ev
