#!/bin/bash
# round 4 session 33: host pool jobs ending on task completion; one fused scan over a chunk's events (programme, bad instance, front-end
# eligibility, partition counts) and the mirror pass reading compact per-instance
# records (written during the range's counting sort) instead of gathering the events --
# front-end / event tests, then the dense-event modes with host phase times, base and new
# alternating on one box
set -u
OUT=gpurun_out/r04s33; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
B=tunebfree_amd/_variants/libtbf_hostbase.so
timeout -k 10 400 python3 -u -m pytest tests -x -v -s -m gpu -k "front or event or dense or program or note" --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|Error" $OUT/tests.log | head -5; tail -2 $OUT/tests.log; st tests $rc
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
timeout -k 10 300 env TBF_LIB=$B TBF_DEBUG_HOST_PHASES=1 python3 -u tools/dense_events.py --out $OUT/base_$i.json > $OUT/base_$i.log 2>&1; st base_$i $?
timeout -k 10 300 env TBF_DEBUG_HOST_PHASES=1 python3 -u tools/dense_events.py --out $OUT/new_$i.json > $OUT/new_$i.log 2>&1; st new_$i $?
done
python3 - <<'PY'
import json
for n in ("base_1", "new_1", "base_2", "new_2"):
    d = json.load(open(f"gpurun_out/r04s33/{n}.json"))
    print(n, [(r["mode"], round(r["ms_per_step"], 3), round(r["host_control_ms_per_step"], 3)) for r in d["rows"]])
PY
