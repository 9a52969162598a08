#!/bin/bash
# round 4 session 25: the play matrix on the device (k_tpl_matrix) -- template tests, then
# the whole GPU suite
set -u
OUT=gpurun_out/r04s25; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
timeout -k 10 300 python3 -u -m pytest tests -x -v -s -m gpu -k "template or matrix" --timeout 240 --timeout-method thread > $OUT/tpl.log 2>&1; rc=$?
grep -E "FAILED|Error|assert|templates \(|device templates" $OUT/tpl.log | head -12; tail -2 $OUT/tpl.log; st tpl $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python3 -u -m pytest tests -x -v -s -m gpu --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|Error" $OUT/tests.log | head -5; tail -2 $OUT/tests.log; st tests $rc
