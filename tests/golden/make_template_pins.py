"""Generate tests/golden/template_pins.json: digests of the tonegen template tables
built by the reference's OWN code -- src/tonegen.cpp's static initOscillators
(writeSamples with its per-sample rand() LSB), initKeyCompTable and initEnvelopes
(random click bursts), reached by oracle/ref_tpl_pin.cpp, which #includes that file
unmodified (`make -C oracle pin`).  Run here, where /root/reference exists; the JSON is
data only (inputs = sample rate, tuning, seed; outputs = SHA-256 of the float32 tables
plus a few sampled values; the play matrix from the reference's compilePlayMatrix) and
pins the oracle's and the product's template builders
on machines without /root/reference.

Cases: the 7 tunings of tests/golden/tunings.json x 48 / 96 kHz, template seed 300 + j
(j = tuning index in sorted order), the frequency table of each from the oracle's
getFrequencies restatement (pinned by the reference's osc.txt fixtures).
"""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))

from orc_bind import load_oracle, load_pin, pin_template  # noqa: E402

KEYS = ("bank", "lens", "wfreq", "attack", "release", "keycomp", "contrib")


def digest(tables):
    out = {k: hashlib.sha256(np.ascontiguousarray(tables[k]).tobytes()).hexdigest() for k in KEYS}
    b = tables["bank"]
    out["bank_size"] = int(b.size)
    out["bank_probe"] = [float(x) for x in b[:: max(1, b.size // 16)][:16]]
    return out


def cases():
    """(tuning, sr, seed, mts128, cfg set name or None)"""
    tun = json.loads((HERE / "tunings.json").read_text())
    names = sorted(tun)
    for sr in (48000.0, 96000.0):
        for j, nm in enumerate(names):
            yield nm, sr, 300 + j, (None if tun[nm] is None else np.array(tun[nm], np.float64)), None
    # the template cfg keys (envelope models / levels / lengths, x-precision; wheel EQ,
    # harmonics, terminal mix, taper, crosstalk lists and levels, contribution floor)
    for k, cfgname in enumerate(("envelopes", "envelopes2", "osc_lists", "osc_models")):
        yield "12TET", 48000.0, 400 + k, None, cfgname
    yield "19TET", 96000.0, 410, np.array(tun["19TET"], np.float64), "osc_lists"


def main():
    orc, pin = load_oracle(), load_pin()
    if pin is None:
        raise SystemExit("oracle/_ref/libtbfpin.so not built (make -C oracle pin)")
    import scenarios as S
    from orc_bind import Cfg
    rows = []
    for nm, sr, seed, m, cfgname in cases():
        cfg = None if cfgname is None else Cfg(orc, S.CFG_SETS[cfgname])
        rows.append({"tuning": nm, "sr": sr, "seed": seed, "cfg": cfgname,
                     **digest(pin_template(pin, orc, sr, m, seed, cfg))})
    (HERE / "template_pins.json").write_text(json.dumps(rows, indent=1) + "\n")
    print(f"wrote template_pins.json: {len(rows)} templates")


if __name__ == "__main__":
    main()
