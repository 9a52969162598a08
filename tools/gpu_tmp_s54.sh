#!/bin/bash
# one-off: TBF_CTL_STREAM=1 (uploads, k_front, k_tgctl on the engine stream): GPU suite under it, same-box A/B
set -u
O=gpurun_out/r05s54; mkdir -p $O
TBF_CTL_STREAM=1 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed $?; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 0 1; do
    TBF_CTL_STREAM=$v timeout -k 10 200 python3 -u tools/dense_events.py --modes every8,dense --steps 8 --warmup 3 > $O/cs${v}_$r.log 2>&1 || { echo $v failed $?; exit 1; }
    echo cs$v $r $(grep mode $O/cs${v}_$r.log | python3 -c "import sys,json; print(' '.join(r['mode']+' '+str(round(r['ms_per_step'],3)) for r in map(json.loads, sys.stdin)))")
  done
done
for v in 0 1; do
  TBF_CTL_STREAM=$v timeout -k 10 400 python3 -u bench.py --steps 8 --warmup 3 > $O/bench$v.json 2> $O/bench$v.err || { echo bench failed $?; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench$v.json')); print('bench cs$v', d['value'], d['ms_per_step'], d.get('steady64_ms'))"
done
