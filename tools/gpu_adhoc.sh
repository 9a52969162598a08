#!/bin/bash
# ad-hoc session: GPU tests (-k filter optional: $1), then the bench with each kernel also timed alone
set -u
OUT=gpurun_out/${TAG:-adhoc}; mkdir -p $OUT; export TMPDIR=/tmp
K=${1:-}
timeout -k 10 600 python3 -u -m pytest tests -x -v -s -m gpu ${K:+-k "$K"} --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" $OUT/tests.log | tail -5; echo "tests rc=$rc"
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 - $OUT/bench.json <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("value %.4g ms/step %.2f err %s exact %s steady64 %.3f" % (d["value"], d["ms_per_step"], d["max_err"], d["bit_exact_frac"], d["steady64"]["ms_per_64_blocks"]))
print({k: round(v["ms_isolated"], 2) for k, v in d["roofline"]["kernels"].items()})
PY
