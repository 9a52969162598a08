#!/bin/bash
# round 4 session 23: steady chunks of up to 512 blocks -- steady / full-size tests, the
# bench at 512- and 256-block steps (twice, alternating; the driver's step counts)
set -u
OUT=gpurun_out/r04s23; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print('value %.4g ms/step %.3f err %s' % (d['value'], d['ms_per_step'], d['max_err']), 'iso', {k: round(v, 3) for k, v in (r['kernels_ms_isolated'] or {}).items()})" $1; }
timeout -k 10 600 python3 -u -m pytest tests -x -v -s -m gpu --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|Error" $OUT/tests.log | head -5; tail -2 $OUT/tests.log; st tests $rc
for i in 1 2 3; do
for b in 512 256; do
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --steps 20 --warmup 5 --blocks $b > $OUT/bench_b${b}_$i.json 2> $OUT/bench_b${b}_$i.err; st b${b}_$i $?
summ $OUT/bench_b${b}_$i.json
done
done
