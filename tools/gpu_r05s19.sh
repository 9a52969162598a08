#!/bin/bash
# host-phase breakdown of the dense-event modes and the steady-chunk penalty per kernel
set -u
OUT=gpurun_out/r05s19; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 env TBF_DEBUG_HOST_PHASES=1 python3 -u tools/dense_events.py --modes every8,dense --steps 3 --warmup 1 > $OUT/dense_phases.log 2> $OUT/dense_phases.err || exit $?
for c in 512 2048; do
	timeout -k 10 300 env TBF_STEADY_CHUNK=$c python3 bench.py --cpu-baseline 0 --check 0 --stage-check 0 --steps 5 --warmup 2 --isolated 2 --steady64 0 > $OUT/chunk$c.json 2> $OUT/chunk$c.err || exit $?
	python3 -c "
import json
d=json.loads([l for l in open('$OUT/chunk$c.json') if l.startswith('{')][-1])
print('chunk $c', '%.4g'%d['value'], '%.2f ms'%d['ms_per_step'], {k:round(v['ms_isolated'],2) for k,v in d['roofline']['kernels'].items()})"
done
grep -v "^chunk" $OUT/dense_phases.err | sort | uniq -c | sort -rn | head -5
grep "stepChunkFront\|threads" $OUT/dense_phases.err | tail -12
