#!/bin/bash
# k_whirl_split auto-selection: parity suite, cfg5 (96 kHz ring of 1024) and 2048 instances
# with each whirl kernel, RT latency
set -u
OUT=gpurun_out/r05s30; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -n 3 $OUT/tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
for sp in 0 1; do
	timeout -k 10 300 env TBF_WHIRL_SPLIT=$sp python3 bench.py --workload cfg5 --cpu-baseline 0 --check 4 --steps 3 --warmup 1 --steady64 0 --isolated 2 > $OUT/cfg5_$sp.json 2>> $OUT/err.log || exit $?
	timeout -k 10 300 env TBF_WHIRL_SPLIT=$sp python3 bench.py --batch 2048 --cpu-baseline 0 --check 4 --steps 5 --warmup 2 --steady64 0 --isolated 2 > $OUT/b2048_$sp.json 2>> $OUT/err.log || exit $?
	for f in cfg5_$sp b2048_$sp; do python3 -c "
import json
d=json.loads([l for l in open('$OUT/$f.json') if l.startswith('{')][-1])
print('$f', '%.4g'%d['value'], '%.2f ms'%d['ms_per_step'], 'err', d['max_err'], 'whirl %.2f'%d['roofline']['kernels']['k_whirl']['ms_isolated'])"; done
	timeout -k 10 300 env TBF_WHIRL_SPLIT=$sp python3 -u tools/rt_latency.py --out $OUT/rt_$sp.json > $OUT/rt_$sp.log 2>&1 || exit $?
	python3 -c "
import json
for r in json.load(open('$OUT/rt_$sp.json'))['rows'][:4]: print('rt split $sp', r['frames'], 'p50 %.3f p99 %.3f' % (r['p50_ms'], r['p99_ms']))"
done
