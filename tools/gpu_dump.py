import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import scenarios as S
from enginerun import engine_run
import tunebfree_amd as T
db = [("param", S.P_DRAWBAR + j, v) for j, v in enumerate([8, 8, 8, 0, 0, 0, 0, 0, 0])]
out = {}
for nb in (3, 8):
    n = 4
    scs = [[(0, k, a, b) for (k, a, b) in db] + [(0, "note", k, 1) for k in S.chord_for(i)] for i in range(n)]
    eng = T.Engine(device=0, chain=1)
    tid = eng.template(seed=7)
    eng.add_instances([tid] * n, [1000 + 17 * i for i in range(n)])
    L, R = engine_run(eng, scs, nb)
    out[f"L{nb}"] = L
    del eng
np.savez(sys.argv[1], **out)
print("saved")
