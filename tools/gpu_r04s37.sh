#!/bin/bash
# round 4 session 37: dense-event modes with 1024- and 512-block steady chunks, alternating
set -u
OUT=gpurun_out/r04s37; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
for i in 1 2; do
timeout -k 10 300 python3 -u tools/dense_events.py --out $OUT/d1024_$i.json > $OUT/d1024_$i.log 2>&1; st d1024_$i $?
timeout -k 10 300 env TBF_STEADY_CHUNK=512 python3 -u tools/dense_events.py --out $OUT/d512_$i.json > $OUT/d512_$i.log 2>&1; st d512_$i $?
done
python3 - <<'PY'
import json
for n in ("d1024_1", "d512_1", "d1024_2", "d512_2"):
    d = json.load(open(f"gpurun_out/r04s37/{n}.json"))
    print(n, [(r["mode"], round(r["ms_per_step"], 3), round(r["host_control_ms_per_step"], 3)) for r in d["rows"]])
PY
