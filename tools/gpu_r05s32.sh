#!/bin/bash
# the front-end tests, then the host phases under dense events
set -u
OUT=gpurun_out/${TAG:-r05s32}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -n 3 $OUT/tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u tools/dense_events.py --modes steady,every8,params,dense --out $OUT/dense.json > $OUT/dense.log 2>&1 || exit $?
python3 -c "
import json
for r in json.load(open('$OUT/dense.json'))['rows']: print('  %-8s %.3f ms  host %.3f ms' % (r['mode'], r['ms_per_step'], r['host_control_ms_per_step']))"
timeout -k 10 300 env TBF_DEBUG_HOST_PHASES=1 python3 -u tools/dense_events.py --modes dense --steps 4 --warmup 2 > /dev/null 2> $OUT/dense_ph.err || exit $?
grep -E "clean|stepChunkFront|threads" $OUT/dense_ph.err | tail -9
