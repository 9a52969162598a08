#!/bin/bash
# stage-buffer footprint vs speed: the bench at 2048-block steps for (steady chunk, stage groups) pairs
set -u
OUT=gpurun_out/${TAG:-groups}; mkdir -p $OUT; export TMPDIR=/tmp
B="--cpu-baseline 0 --check 0 --stage-check 0 --steps 10 --warmup 3 --isolated 0 --steady64 0"
for cfg in "$@"; do
	c=${cfg%%:*}; g=${cfg#*:}; name="c${c}_g${g//,/}"
	timeout -k 10 300 env TBF_STEADY_CHUNK=$c TBF_PIPE_GROUPS=$g python3 bench.py $B > $OUT/$name.json 2> $OUT/$name.err; rc=$?
	[ $rc -ne 0 ] && { echo "$name rc=$rc"; exit $rc; }
	python3 -c "
import json
d=json.loads([l for l in open('$OUT/$name.json') if l.startswith('{')][-1])
print('$name', '%.4g'%d['value'], '%.2f ms'%d['ms_per_step'])"
done
