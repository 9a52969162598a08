#!/bin/bash
# one-off: k_mixpre's output mid1 in three sets (k_mixpre of chunk c no longer waits for chunk c-2's k_rv_post): suite, same-box A/B
set -u
O=gpurun_out/r05s60; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed $?; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 2 3; do
    TBF_MID1_SETS=$v timeout -k 10 400 python3 -u bench.py --cpu-baseline 0 --steps 20 --warmup 5 > $O/b${v}_$r.json 2> $O/b${v}_$r.err || { echo bench failed $?; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/b${v}_$r.json') if l.startswith('{')][-1]); print('sets $v run $r', round(d['value']/1e9,3), round(d['ms_per_step'],2), round(d['steady64']['ms_per_64_blocks'],3), d['max_err'])"
  done
done
