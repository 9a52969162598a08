#!/bin/bash
# round 4 session 8: device front end with parameter events; phase clocks at 256 blocks; dense events
set -u
OUT=gpurun_out/r04s8; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
timeout -k 10 600 python3 -u -m pytest tests -x -v -s -m gpu -k "front_end or steady or threaded" --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; st tests $?
tail -3 $OUT/tests.log
timeout -k 10 500 python3 -u tools/dense_events.py --out $OUT/dense_events.json > $OUT/dense.log 2>&1; st dense $?
tail -6 $OUT/dense.log
bash tools/gpu_session.sh r04s8 prof
