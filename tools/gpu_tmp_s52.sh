#!/bin/bash
# one-off: A/B of the k_tgctl / k_front / k_tonegen dense-path changes: GPU suite, dense events, bench
set -u
O=gpurun_out/${TAG:-r05s52}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed $?; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u tools/dense_events.py --modes steady,every8,dense --steps 8 --warmup 3 > $O/de.log 2>&1 || { echo de failed $?; exit 1; }
grep mode $O/de.log | python3 -c "import sys,json; [print(r['mode'], round(r['ms_per_step'],3)) for r in map(json.loads, sys.stdin)]"
timeout -k 10 400 python3 -u bench.py --steps 8 --warmup 3 > $O/bench.json 2> $O/bench.err || { echo bench failed $?; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'])"
