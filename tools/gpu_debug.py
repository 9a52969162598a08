"""Ad-hoc GPU parity localisation (developer tool; uses the oracle as checker)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import scenarios as S
from enginerun import compare, engine_run, oracle_run
from orc_bind import load_oracle, Template
import tunebfree_amd as T

lib = load_oracle()

def run(name, scen_fn, chain, n=4, nb=8, idx=2):
    eng = T.Engine(device=0, chain=chain)
    tid = eng.template(seed=7)
    seeds = [1000 + 17 * i for i in range(n)]
    eng.add_instances([tid] * n, seeds)
    tpl = Template(lib, seed=7)
    scens = [scen_fn(i) for i in range(n)]
    L, R = engine_run(eng, scens, nb)
    ref = oracle_run(lib, tpl, seeds, scens, nb, chain=1 if chain == 1 else 0)
    r = ref[idx]
    err, ex = compare(L, r)
    bad = np.nonzero(L.view(np.uint32) != r.view(np.uint32))
    first = (bad[0][0], bad[1][0]) if len(bad[0]) else None
    print(f"{name}: err={err:.3g} exact={ex:.4f} first={first}", flush=True)
    if first:
        i, s = first
        print("   gpu", L[i, s:s+4], "orc", r[i, s:s+4])
        blocks = sorted(set((bad[1] // 128).tolist()))[:10]
        print("   bad blocks", blocks, "per-block count", [int(np.sum(bad[1] // 128 == b)) for b in blocks[:5]])

db = [("param", S.P_DRAWBAR + j, v) for j, v in enumerate([8, 8, 8, 0, 0, 0, 0, 0, 0])]
def mk(extra):
    return lambda i: [(0, k, a, b) for (k, a, b) in db + extra] + [(0, "note", k, 1) for k in S.chord_for(i)]

run("plain", mk([]), 1)
run("vib V1", mk([("param", S.P_VIBRATO_TYPE, 0), ("param", S.P_VIBRATO, 1)]), 1)
run("vib C3", mk([("param", S.P_VIBRATO_TYPE, 5), ("param", S.P_VIBRATO, 1)]), 1)
run("perc", mk([("param", S.P_PERC, 1)]), 1)
run("od tap", S.bench_scenario, 2, idx=3)
run("rv tap", S.bench_scenario, 3, idx=4)
run("full", S.bench_scenario, 0, idx=0)
