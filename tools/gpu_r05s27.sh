#!/bin/bash
# k_whirl_split: GPU parity suite, then the bench with and without it
set -u
OUT=gpurun_out/${TAG:-r05s27}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -n 3 $OUT/tests.log; echo "tests rc=$rc"; [ $rc -ge 124 ] && exit $rc
B="--cpu-baseline 0 --check 4 --stage-check 0 --steps 5 --warmup 2 --steady64 0"
for sp in 1 0; do
	timeout -k 10 300 env TBF_WHIRL_SPLIT=$sp python3 bench.py $B > $OUT/split$sp.json 2> $OUT/split$sp.err || exit $?
	python3 -c "
import json
d=json.loads([l for l in open('$OUT/split$sp.json') if l.startswith('{')][-1])
print('split $sp', '%.4g'%d['value'], '%.2f ms'%d['ms_per_step'], 'err', d['max_err'], {k:round(v['ms_isolated'],2) for k,v in d['roofline']['kernels'].items()})"
done
