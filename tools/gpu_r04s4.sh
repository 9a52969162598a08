#!/bin/bash
# round 4 session 4: steady chunks (TBF_STEADY_CHUNK) -- tests, bench at 64 / 128 / 256 blocks per step
set -u
OUT=gpurun_out/r04s4; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
timeout -k 10 900 python3 -u -m pytest tests -x -v -s -m gpu --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; st tests $?
tail -3 $OUT/tests.log
for b in 64 128 256; do
  timeout -k 10 300 python3 bench.py --cpu-baseline 0 --blocks $b --isolated 1 > $OUT/bench_$b.json 2> $OUT/bench_$b.err; st bench_$b $?
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(sys.argv[2], 'value %.4g ms/step %.3f err %s' % (d['value'], d['ms_per_step'], d['max_err']), 'kern', {k: round(v, 3) for k, v in r['kernels_ms_per_launch'].items()}, 'iso', {k: round(v, 3) for k, v in (r['kernels_ms_isolated'] or {}).items()})" $OUT/bench_$b.json $b
done
echo done
