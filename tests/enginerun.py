"""Drive the HIP engine and the oracle with the same per-instance event scripts."""
from __future__ import annotations

import numpy as np

import scenarios as S


def engine_run(eng, scens, nblocks, tids=None):
    """scens: list (one per instance) of scenario event lists; events land at block
    boundaries exactly like the reference's MIDI (b_synth/lv2.cpp:1130-1134).
    ("retune", j, 0) retunes the instance to template tids[j] (tbf_instance_retune);
    ("control", name, value) calls a MIDI control function (tbf_midi_control)."""
    bounds = {0, nblocks}
    for sc in scens:
        bounds.update(b for (b, *_r) in sc if b < nblocks)
    bounds = sorted(bounds)
    outL, outR = [], []
    for s, e in zip(bounds[:-1], bounds[1:]):
        for i, sc in enumerate(scens):
            for (b, kind, a, v) in sc:
                if b != s:
                    continue
                if kind == "note":
                    eng.note(i, a, v)
                elif kind == "retune":
                    eng.retune(i, tids[a])
                elif kind == "control":
                    assert eng.midi_control(i, a, v)
                else:
                    eng.set_param(i, a, v)
        L, R = eng.render(e - s)
        outL.append(L)
        outR.append(R)
    return np.concatenate(outL, axis=1), np.concatenate(outR, axis=1)


def oracle_run(lib, tpl, seeds, scens, nblocks, chain=0, templates=None):
    from orc_bind import Chain
    Ls, Rs, As, Bs, Cs = [], [], [], [], []
    for seed, sc in zip(seeds, scens):
        ch = Chain(lib, tpl, seed)
        ch.chain(1 if chain == 1 else 0)
        L, R, A, B, C = S.run(ch, sc, nblocks, stages=True, templates=templates)
        Ls.append(L); Rs.append(R); As.append(A); Bs.append(B); Cs.append(C)
    return [np.stack(x) for x in (Ls, Rs, As, Bs, Cs)]


def compare(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))
    exact = float(np.mean(a.view(np.uint32) == b.view(np.uint32)))
    return float(d.max()) if d.size else 0.0, exact
