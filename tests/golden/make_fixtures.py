"""Generate the committed fixtures under tests/golden/ (run here, where
/root/reference exists; the outputs are data only).

  tunings.json               128-note frequency tables of the reference's tests:
                             12TET (MTS-ESP no-master), 19TET / Bohlen-Pierce / p4 /
                             bagpipe4 (tables embedded in src/tuning.cpp doctests),
                             5TET / duodene (tests/regression_test_data/*.scl mapped
                             with note 60 = 261.62556530059874 Hz, period from the scl)
  regression_test_data.tar.xz  the reference's DEBUG_TONEGEN_OSC fixture files
  ref_vectors.npz            reference-compiled chain outputs (oracle/_ref) for the
                             golden scenarios, with per-stage taps
"""
import json
import lzma
import re
import subprocess
import sys
import tarfile
from fractions import Fraction
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
REF = Path("/root/reference")
sys.path.insert(0, str(ROOT / "tests"))


def tuning_tables():
    src = (REF / "src/tuning.cpp").read_text()
    tabs = {}
    for m in re.finditer(r'TEST_CASE\("Testing (?:inferPeriod|extendFrequencies) ([^"]+)"\)\s*\{\s*double frequency\[(\d+)\] = \{(.*?)\};', src, re.S):
        name = m.group(1).split()[0].replace(".scl", "")
        vals = [float(v) for v in re.findall(r"[-0-9.eE+]+", m.group(3))]
        tabs.setdefault(name, vals[:128])
    return tabs


def scl_freqs(path, base=261.62556530059874, note=60):
    lines = [l.strip() for l in Path(path).read_text().splitlines() if not l.strip().startswith("!")]
    n = int(lines[1])
    steps = []
    for l in lines[2:2 + n]:
        tok = l.split()[0]
        if "/" in tok or "." not in tok:
            steps.append(float(Fraction(tok)))
        else:
            steps.append(2.0 ** (float(tok) / 1200.0))
    period = steps[-1]
    ratios = [1.0] + steps[:-1]
    out = []
    for k in range(128):
        d = k - note
        o, r = divmod(d, n)
        out.append(base * period ** o * ratios[r])
    return out


def main():
    tabs = tuning_tables()
    t = {"12TET": None,
         "19TET": tabs["19TET"],
         "Bohlen-Pierce": tabs["Bohlen-Pierce"],
         "p4": tabs["p4"],
         "bagpipe4": tabs["bagpipe4"],
         "5TET": scl_freqs(REF / "tests/regression_test_data/5TET/ED2-05.scl"),
         "duodene": scl_freqs(REF / "tests/regression_test_data/duodene/duodene.scl")}
    (HERE / "tunings.json").write_text(json.dumps(t, indent=0))
    with tarfile.open(HERE / "regression_test_data.tar.xz", "w:xz") as tf:
        tf.add(REF / "tests/regression_test_data", arcname="regression_test_data")
    print("wrote tunings.json, regression_test_data.tar.xz")


if __name__ == "__main__":
    main()
