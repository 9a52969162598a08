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


def run(chain, scenario, nblocks, stages=False):
    """Apply events at block boundaries and render; returns concatenated arrays."""
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
            else:
                chain.param(a, v)
        outs.append(chain.render(e - s, stages=stages))
    return [np.concatenate(x) for x in zip(*outs)]
