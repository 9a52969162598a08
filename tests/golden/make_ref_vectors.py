"""Generate tests/golden/ref_vectors.npz: outputs of the reference's OWN translation
units (oracle/_ref/libtbfref.so, compiled from /root/reference/src by `make -C oracle
ref`) for fixed golden scenarios, with every stage tap.  Run here, where
/root/reference exists; the file is data only (inputs = the case table below,
outputs = float32 streams) and lets the oracle and the GPU engine be checked against
the reference on machines without /root/reference.

Per case the npz holds <case>/L, /R (whirlProc3 outputs), /A (oscGenerateFragment
output), /B (preamp output), /C (reverb output), and `cases` = the JSON case table.
The tonegen template (wave bank, play matrix, envelopes) of a case is built from
(sr, tuning, tpl_seed) -- initToneGenerator itself is unbuildable here.
"""
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))

import scenarios as S  # noqa: E402
from orc_bind import Chain, Template, load_oracle, load_ref  # noqa: E402

# name, sr, tuning (tunings.json key or None = 12-TET no-master), tpl_seed, inst_seed,
# scenario (fn, arg), nblocks, chain (0 full, 1 tonegen only)
CASES = [
    ("bench48", 48000.0, None, 7, 1011, ("bench", 3), 48, 0),
    ("events48", 48000.0, None, 7, 1005, ("events", 5), 72, 0),
    ("tonegen48", 48000.0, None, 3, 77, ("bench_tg", 1), 40, 0),
    ("events44_19tet", 44100.0, "19TET", 5, 4242, ("events", 2), 72, 0),
    ("bench96_p4", 96000.0, "p4", 11, 9, ("bench", 17), 40, 0),
    ("random96_bagpipe4", 96000.0, "bagpipe4", 13, 31, ("random", 3), 40, 0),
    # parameter sweep (scenarios.sweep_scenario): overdrive character, reverb mix, percussion
    # variants, clusters, pedal keys, rotary stop <-> fast
    ("sweep48_0", 48000.0, None, 7, 2100, ("sweep", 0), 72, 0),
    ("sweep48_1", 48000.0, None, 7, 2101, ("sweep", 1), 72, 0),
    ("sweep48_2", 48000.0, None, 7, 2102, ("sweep", 2), 72, 0),
    ("sweep48_3", 48000.0, None, 7, 2103, ("sweep", 3), 72, 0),
    ("sweep44_5", 44100.0, "duodene", 9, 2105, ("sweep", 5), 72, 0),
    ("sweep96_6", 96000.0, "5TET", 3, 2106, ("sweep", 6), 48, 0),
    # drawbar / routing / percussion changes with no key event in the block
    ("reroute48_1", 48000.0, None, 7, 2201, ("reroute", 1), 56, 0),
]


def scenario(kind, i):
    if kind == "bench":
        return S.bench_scenario(i)
    if kind == "events":
        return S.event_scenario(i)
    if kind == "bench_tg":
        return S.bench_scenario(i, full=False) + [(20, "note", 70, 1), (30, "param", S.P_PERC, 1)]
    if kind == "random":
        return S.random_drawbar_scenario(i)
    if kind == "sweep":
        return S.sweep_scenario(i)
    if kind == "reroute":
        return S.reroute_scenario(i)
    raise ValueError(kind)


def main():
    orc, ref = load_oracle(), load_ref()
    if ref is None:
        raise SystemExit("oracle/_ref/libtbfref.so not built (make -C oracle ref)")
    tunings = json.loads((HERE / "tunings.json").read_text())
    out, table = {}, []
    for (name, sr, tun, tseed, iseed, (kind, arg), nb, chain) in CASES:
        m = None if tun is None else np.array(tunings[tun], np.float64)
        tpl = Template(orc, sr=sr, mts128=m, seed=tseed)
        ch = Chain(ref, tpl, iseed, ref=True)
        ch.chain(chain)
        L, R, A, B, C = S.run(ch, scenario(kind, arg), nb, stages=True)
        for k, v in zip("LRABC", (L, R, A, B, C)):
            out[f"{name}/{k}"] = v.astype(np.float32)
        table.append({"name": name, "sr": sr, "tuning": tun, "tpl_seed": tseed, "inst_seed": iseed,
                      "scenario": [kind, arg], "nblocks": nb, "chain": chain})
    out["cases"] = np.array(json.dumps(table))
    np.savez_compressed(HERE / "ref_vectors.npz", **out)
    print(f"wrote ref_vectors.npz: {len(table)} cases")


if __name__ == "__main__":
    main()
