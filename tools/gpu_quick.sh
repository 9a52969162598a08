#!/bin/bash
# tools/gpu_quick.sh TAG -- parity tests, stage profile and a short bench on the GPU box.
set -u
TAG=${1:-dev}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -m pytest tests -x -q -m gpu > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/prof_stages.py > "$OUT/prof.log" 2>&1
rc=$?; cat "$OUT/prof.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --cpu-baseline 0 > "$OUT/bench.log" 2>&1
rc=$?; grep '^{' "$OUT/bench.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH', d['value'], d['ms_per_step'], d['max_err'], d['bit_exact_frac'])"
exit $rc
