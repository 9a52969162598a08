#!/bin/bash
# k_whirl_split without spills (4 waves per SIMD, 128 VGPRs) against k_whirl, at 2048 and 4096 instances
set -u
OUT=gpurun_out/r05s29; mkdir -p $OUT; export TMPDIR=/tmp
B="--cpu-baseline 0 --check 0 --stage-check 0 --steps 3 --warmup 1 --steady64 0 --isolated 2"
for cfg in "4096 0 base" "4096 1 whs4" "2048 0 base" "2048 1 whs4" "2048 1 base"; do
	set -- $cfg; b=$1; sp=$2; lib=$3
	L=tunebfree_amd/libtbf.so; [ $lib != base ] && L=tunebfree_amd/_variants/libtbf_$lib.so
	timeout -k 10 300 env TBF_LIB=$L TBF_WHIRL_SPLIT=$sp python3 bench.py --batch $b $B > $OUT/r_${b}_${sp}_${lib}.json 2> $OUT/err.log || exit $?
	python3 -c "
import json
d=json.loads([l for l in open('$OUT/r_${b}_${sp}_${lib}.json') if l.startswith('{')][-1])
print('batch $b split $sp lib $lib', '%.2f ms'%d['ms_per_step'], 'whirl %.2f'%d['roofline']['kernels']['k_whirl']['ms_isolated'])"
done
