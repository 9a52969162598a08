#!/bin/bash
# round 4 session 22: host front end walks per-range event copies, key bitset kept
# incrementally -- front-end / event tests, dense-event modes with host phase times
set -u
OUT=gpurun_out/r04s22; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
timeout -k 10 600 python3 -u -m pytest tests -x -v -s -m gpu -k "front or event or dense or program or note" --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|Error" $OUT/tests.log | head -5; tail -2 $OUT/tests.log; st tests $rc
timeout -k 10 500 env TBF_DEBUG_HOST_PHASES=1 python3 -u tools/dense_events.py --out $OUT/dense_events.json > $OUT/dense.log 2>&1; st dense $?
grep -E "^\{|partition" $OUT/dense.log | tail -12
