#!/bin/bash
# ablation timings: the default bench (no parity check) on the in-tree library and on each
# variant named as an argument (tunebfree_amd/_variants/libtbf_NAME.so); timing experiments
# only -- a variant's output is wrong by construction
set -u
OUT=gpurun_out/${TAG:-abl}; mkdir -p $OUT; export TMPDIR=/tmp
B="--cpu-baseline 0 --check 0 --stage-check 0 --steps 5 --warmup 2 --steady64 0"
for v in base "$@"; do
	if [ $v = base ]; then L=tunebfree_amd/libtbf.so; else L=tunebfree_amd/_variants/libtbf_$v.so; fi
	timeout -k 10 300 env TBF_LIB=$L python3 bench.py $B > $OUT/$v.json 2> $OUT/$v.err; rc=$?
	echo "$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
	python3 -c "
import json,sys
d=json.loads([l for l in open('$OUT/$v.json') if l.startswith('{')][-1])
print('$v', '%.4g'%d['value'], '%.2f ms'%d['ms_per_step'], {k:round(v['ms_isolated'],2) for k,v in d['roofline']['kernels'].items()})"
done
